// pmmg_hip.hip — MI355X (gfx950) old->new mesh transfer: locate every new
// vertex in the background mesh and interpolate metric + fields (fp64).
//
// Replaces, behind the C-ABI of include/parmmg_hip.h, the per-group body of
// PMMG_interpMetricsAndFields (reference src/interpmesh_pmmg.c:477-741):
//   PMMG_locatePointVol      src/locate_pmmg.c:786-883     -> k_vol<layout> (fp32 filter walk + exact
//                                                             acceptance + interpolation), k_vol_walk_exact
//   PMMG_interp4bar_*        src/interpmesh_pmmg.c:206-270 -> vol_slot / vol_interp_packed in k_vol (pmmg_vol.hpp)
//   PMMG_locatePointBdy      src/locate_pmmg.c:587-723     -> k_bdy (locate + interpolate)  (pmmg_bdy.hpp)
//   exhaustive / closest     src/locate_pmmg.c:477-515, 737-770 -> k_*_exhaust_accept, k_*_exhaust_closest
//                                                             (pmmg_fallback.hpp)
// Device arithmetic: pmmg_device.hpp; preparation and query order:
// pmmg_prep.hpp.
//
// Pipeline of one pmmg_hip_locate_interp (no host synchronisation inside):
//   main stream     reset, coherence test, frame, volume seeds | query order
//                   (Morton bins or stable class compaction, chosen on the
//                   device) | fp32 filter walk + exact acceptance | exact
//                   continuation | interpolation | join | fallbacks
//   surface stream  (after the order) surface seeds, node->tria CSR, k_bdy
#include <hip/hip_ext.h> // hipExtLaunchKernelGGL: events recorded by the kernel dispatch itself
#include <hip/hip_runtime.h>
#ifdef PMMG_HIP_MEASURE
#include <rocprim/device/device_radix_sort.hpp> // the brick renumbering's sort (measurement build)
#endif

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "pmmg_device.hpp"
#include "pmmg_prep.hpp"
#ifdef PMMG_HIP_MEASURE
#include "pmmg_brick.hpp" // measurement build only
#endif
#include "pmmg_sort.hpp"
#include "pmmg_vol.hpp"
#include "pmmg_bdy.hpp"
#include "pmmg_fallback.hpp"
#include "pmmg_snapshot.hpp"
#include "pmmg_quality.hpp"
#include "pmmg_comm.hpp"

using namespace pmmg;

namespace {

// ---------------------------------------------------------------- slot layouts

typedef void (*VolFn)(Bg, const Frame *, const unsigned long long *, int, const double *, const uint8_t *,
                      const int *, const double *, int, ContEntry *, DevStats *, Slots, int *, int8_t *, int,
                      const int *, int, int, int, LocBuf, int, ContArgs);
typedef void (*InterpFn)(LocBuf, const int *, const DevStats *, int, Slots, const int *, int, int, int);

// the split stage's walk kernel: the locate-only layout, writing located records
constexpr VolFn kVolWalk = k_vol<0, 0, 0, 0, 0, 0, 0>;

struct LayoutEntry {
  int c[6];
  VolFn fn;         // one array per solution (the reference's layout)
  VolFn fn_packed;  // packed per-vertex records, one pass (null: layout not packable)
  VolFn fn_packed2; // the same in two passes over the record halves (null: not splittable)
  InterpFn ifn, ifn_packed, ifn_packed2; // the split stage's interpolation kernels, same three forms
};

template <int NP, int A, int B, int C, int D, int E, int F>
constexpr VolFn packed_fn() {
  using L = PackedLayout<A, B, C, D, E, F>;
  if constexpr (L::valid() && L::passes_ok(NP)) return k_vol<NP, A, B, C, D, E, F>;
  else return nullptr;
}
template <int NP, int A, int B, int C, int D, int E, int F>
constexpr InterpFn packed_ifn() {
  using L = PackedLayout<A, B, C, D, E, F>;
  if constexpr (L::valid() && L::passes_ok(NP)) return k_vol_interp<NP, A, B, C, D, E, F>;
  else return nullptr;
}

#define PMMG_LAYOUT(a, b, c, d, e, f)                                                                    \
  {{a, b, c, d, e, f}, k_vol<0, a, b, c, d, e, f>, packed_fn<1, a, b, c, d, e, f>(),                    \
   packed_fn<2, a, b, c, d, e, f>(), k_vol_interp<0, a, b, c, d, e, f>, packed_ifn<1, a, b, c, d, e, f>(), \
   packed_ifn<2, a, b, c, d, e, f>()}
// common slot layouts (metric first): aniso metric + scalar/vector/tensor
// (BASELINE cfg3/cfg4, libexamples cube-solphys.sol), iso metric + scalars
// (cfg2, cfg5), metric only; anything else runs the runtime-layout variant
const LayoutEntry kLayouts[] = {
    PMMG_LAYOUT(6, 1, 3, 6, 0, 0), PMMG_LAYOUT(6, 1, 3, 6, 1, 0), PMMG_LAYOUT(1, 1, 0, 0, 0, 0),
    PMMG_LAYOUT(1, 1, 1, 1, 1, 1), PMMG_LAYOUT(1, 1, 1, 0, 0, 0), PMMG_LAYOUT(6, 0, 0, 0, 0, 0),
    PMMG_LAYOUT(1, 0, 0, 0, 0, 0), PMMG_LAYOUT(6, 1, 0, 0, 0, 0), PMMG_LAYOUT(1, 1, 3, 6, 0, 0),
    PMMG_LAYOUT(0, 0, 0, 0, 0, 0), // locate only (no metric, no field)
};
#undef PMMG_LAYOUT

// passes: packed records' gather passes (1 or 2; the other is taken when the
// layout allows only it; 0 = by the record's size: two above 8 doubles, where
// one pass holds the whole record in registers — cfg4's 16 doubles: 168
// VGPRs, 3 waves per SIMD, 4.42 ms per step against 4.18 in two passes, r05d)
struct VolPick {
  VolFn fn;     // the fused kernel (walk + exact test + interpolation)
  InterpFn ifn; // the split stage's interpolation kernel (after kVolWalk)
};
VolPick pick_layout(const Slots &S, int passes = 0) {
  for (const LayoutEntry &e : kLayouts) {
    int n = 0;
    while (n < 6 && e.c[n] > 0) n++;
    if (n != S.n) continue;
    bool ok = true;
    for (int j = 0; j < n; j++) ok = ok && (S.s[j].code == e.c[j]);
    if (!ok) continue;
    if (!S.rec) return {e.fn, e.ifn};
    if (passes == 0) {
      int k = 0;
      for (int j = 0; j < n; j++) k += e.c[j];
      passes = k > 8 ? 2 : 1;
    }
    VolFn a = passes == 2 ? e.fn_packed2 : e.fn_packed, b = passes == 2 ? e.fn_packed : e.fn_packed2;
    InterpFn ia = passes == 2 ? e.ifn_packed2 : e.ifn_packed, ib = passes == 2 ? e.ifn_packed : e.ifn_packed2;
    return {a ? a : b, ia ? ia : ib};
  }
  if (S.rec) return {nullptr, nullptr};
  return {k_vol<0, -1, 0, 0, 0, 0, 0>, k_vol_interp<0, -1, 0, 0, 0, 0, 0>};
}


// the slot layouts the packed-record interpolation is compiled for
bool packed_supported(int met_size, int nfield, const int *fsize) {
  Slots S{};
  S.rec = reinterpret_cast<const double *>(16);
  if (met_size) S.s[S.n++].code = met_size;
  for (int j = 0; j < nfield && S.n < kMaxSlot; j++) S.s[S.n++].code = fsize[j];
  return pick_layout(S).fn != nullptr;
}

#ifdef PMMG_HIP_MEASURE
// measurement build, PMMG_HIP_SETORDER=1: the query order also written to
// the stats by a one-thread kernel on the main stream, as up to r03ad (the
// volume kernel now takes it as an argument: one launch less between the seed
// grid and the volume kernel)
__global__ void k_set_order(DevStats *st, int sorted, int bits) {
  st->sorted = sorted;
  st->bin_bits = bits;
}
#endif

} // namespace

// ================================================================ host side

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};

enum {
  EV_START, EV_FRAME, EV_PREP, EV_ORDER, EV_VOL0, EV_WALK, EV_VOL, EV_JOIN, EV_END, EV_BDY0, EV_BDY1, EV_RESET,
  EV_SB0, EV_ORDER2, EV_SRFSEED, EV_FILL, EV_BDYFB, EV_QUANT, EV_COUNT
};

struct pmmg_hip_ctx {
  int device = 0;
  int options = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr; // surface branch, concurrent with the volume walk
  hipStream_t stream3 = nullptr; // Morton binning of a call whose order is decided on the device (created at the
                                 // first such call), beside the input order's surface list on stream2
  hipStream_t stream_f = nullptr; // a large call's seed-grid refill, right after the volume kernel, beside the
                                  // main stream's tail (created at the first such call)
  hipStream_t stream2_hi = nullptr; // measurement build, PMMG_HIP_SRFPRIO=1: the same at the highest priority,
  bool srf_prio = false;            // for calls of >= kSmallGroup queries (see run_device)
  char err[512] = {0};
  Bg bg{};
  int met_size = 0;
  int nfield = 0;
  std::vector<int> fsize;
  std::vector<const double *> fin;
  const double *met = nullptr;
  const double *rec = nullptr; // packed per-vertex solution records (set_solutions_packed), else null
  int rstride = 0;             // their stride in doubles
  // owned copies for PMMG_HIP_HOST inputs
  DevBuf o_xyz, o_tetv, o_adja, o_triv, o_adjt, o_met, o_rec;
  std::vector<DevBuf> o_f;
  // work buffers
  DevBuf frame, stats, grid, sgrid, order_v, order_b, cont, xq;
  DevBuf cohd;                            // the coherence test's sampled distances (k_bbox)
  DevBuf axh;                             // per-axis histograms of the seed grid map (k_quantize)
  DevBuf bkeys, bkeys2, bvals, bvals2;    // Morton binning: keys and ids, ping-ponged by the radix sort
  DevBuf rs_hist, rs_csum;                // the radix sort's digit table and its scan's chunk sums
  // PMMG_HIP_BRICK (measurement only, pmmg_brick.hpp): the background renumbered by bricks
  DevBuf brk_k, brk_k2, brk_v, brk_v2, brk_vinv, brk_tinv, brk_xq, brk_xyz, brk_sol, brk_rec, brk_tmp;
  int brick = 0;
  int set_order = 0; // test-only PMMG_HIP_SETORDER=1 (see k_set_order)
  int no_fb = 0;     // measurement build: PMMG_HIP_NOFB
  int stream3_mode = 1; // the binning's own stream: 1 created at the first auto-order call, 2 with the context,
                        // 0 none (measurement build: PMMG_HIP_STREAM3)
  int srf_solo = -1; // the surface branch waits for the seed grid: -1 in calls of >= kSmallGroup queries (r04zo,
                     // cfg4: the seed grid ran at 455 instead of 261 us beside k_bdy; step 4.24 -> 4.13 ms,
                     // Mmg-like 5.01 -> 4.93, shuffled =), 1 always, 0 never (PMMG_HIP_SRFSOLO)
  // the seed grids left clean by the previous call (its last kernels refill
  // them while the other stream finishes): k_reset skips what is clean
  void *grid_clean_p = nullptr, *sgrid_clean_p = nullptr;
  long long grid_clean_n = 0, sgrid_clean_n = 0;
  DevBuf qs;                              // volume query coordinates in processing order (Morton path)
  DevBuf cls_cnt;                         // per-block class counts (surface list compaction)
  DevBuf oflag;                           // the coherence test's {sorted, bin_bits} on the device
  DevBuf qmin;                               // tetra quality minimum (pmmg_hip_tetra_qual)
  DevBuf fb_vol, fb_bdy, best, nac, cres, bbest, bnac, bcres; // exhaustive searches: fallback lists, lowest
  DevBuf fbp_vol, fbp_bdy; // accepting element, unaccepted lists, closest results and range minima (FbPart)
  DevBuf fbg_vol_c, fbg_vol_u, fbg_vol_i, fbg_bdy_c, fbg_bdy_u, fbg_bdy_i; // the lists' query grids
  // host-mode staging
  DevBuf h_xyz, h_cls, h_met, h_elem, h_hit;
  std::vector<DevBuf> h_f;
  hipEvent_t ev[EV_COUNT] = {};
  bool pending = false;
  // host-mode transfers: two pinned staging buffers, filled / drained by a
  // small pool of host threads while the DMA engine moves the other one
  void *stage[2] = {nullptr, nullptr};
  void *stage_dev[2] = {nullptr, nullptr}; // their device addresses (kernel downloads)
  hipEvent_t stage_ev[2] = {};
  int stage_i = 0;
  struct Pool *pool = nullptr;
  DevBuf o_tet4; // device copy of a host tetv (input of the device adjacency)
  SnapCache snap_cache; // the snapshot kernels' scratch (pmmg_snapshot.hip)
  // host mode: the device-built background (adjacency, boundary trias) runs
  // on `stream` in a host thread while set_solutions' uploads go through
  // `cstream` (the DMA engine works beside the snapshot kernels); every other
  // entry point joins it first (snap_join)
  hipStream_t cstream = nullptr;
  std::thread snap;
  int snap_ok = 1;
  int verbose = 0; // PMMG_HIP_VERBOSE: host-mode transfer timings on stderr
  int tpc = 8;        // background tetra per volume seed cell (PMMG_HIP_TPC)
  int seed_lanes = 4;  // sampled tetra per seed run of 4 records (PMMG_HIP_SEEDLANES, 1..4)
  int seed_v0 = 0;     // measurement build, PMMG_HIP_SEEDV0=1: a sample's first vertex instead of its centroid
  int pack_passes = 0; // packed records gathered in 1 or 2 passes over the record (PMMG_HIP_PACKPASS; 0: by size)
  int bbox_stride = 64;  // the frame's bbox samples np / n vertices (PMMG_HIP_BBOX; r03o: 64 instead of 16 and
  int hist_stride = 256; // 256 instead of 64 for the axis histograms: preparation -0.15 ms at cfg4, same walks)
  int bdy_bpx = 512;     // k_bdy blocks per XCD at most (PMMG_HIP_BDYBPX), in blocks of kBlock threads
  int bdy_wave = 0;      // k_bdy in one-wave blocks (PMMG_HIP_BDYWAVE)
  int ev_vol0 = EV_VOL0, ev_vol = EV_VOL; // the events that open / close the call's volume stage (collect_stats)
  int quant_side = 0;    // a large call's fixed-point copy beside the seed grid (PMMG_HIP_QUANTSIDE)
  int fuse_cont = 1;     // the exact continuation inside the volume kernel (PMMG_HIP_FUSECONT=0: the list and
                         // k_vol_walk_exact, as before r06)
  int host_order = 1;    // a large auto-order call reads the coherence test's decision on the host after k_bbox
                         // and enqueues that order's kernels only (PMMG_HIP_HOSTORDER=0: both, gated on the
                         // device, as before r06)
  int *flag_host = nullptr;     // (pinned, coherent: k_bbox's last block writes the decision here too)
  int *flag_host_dev = nullptr; // (its device address)
  int bdy_dyn = 0;       // k_bdy: waves claim work from per-XCD counters (PMMG_HIP_BDYDYN=1; r03y: the claiming
                         // waves slowed the volume kernel beside them, 8-way rank 0.70 -> 0.64 ms static)
  int srf_g = 0;         // test-only PMMG_HIP_SRFG: the surface seed grid's cells per axis (1: one seed for all)
  int srf_mult = 8;      // the surface seed grid has srf_mult * nt / 2 cells (PMMG_HIP_SRFMULT; r03r at cfg4: 1 /
                         // 8 / 32 -> 7.4 / 3.9 / 2.7 steps per surface point, surface branch 0.446 / 0.403 /
                         // 0.399 ms: a surface grid sized like a volume grid left ~33 trias per occupied cell)
  int bin_bits = kBinBitsCoherent; // Morton bits per axis of the binning keys when the order is forced (1..7,
                                    // PMMG_HIP_BINBITS; auto mode: the coherence test picks)
  int bin_qs = 0;       // the binning copies the volume queries' coordinates in processing order (PMMG_HIP_BINQS=1;
                        // r03: -0.5 ms in the walk on a shuffled numbering, +1 ms in the binning)
  int maxstep = 1024; // longer walks go to the exhaustive kernels (PMMG_HIP_MAXSTEP; the reference caps at ne).
                      // r05: 4096 -> 1024; a walk that long cycles along a concave boundary (carried cfg4
                      // iteration: 2644 queries at the cap, all then accepted by the exhaustive search; the
                      // longest legitimate walk seen is 302 steps, cfgG)
  int fanmax = kFanMax;    // cone fans longer than this take the O(nt) scan (test-only PMMG_HIP_FANMAX)
  int pad = 0;           // measurement build, PMMG_HIP_PAD: extra VALU / L1 work per walk step (k_vol)
  int xcd_run = 64;      // k_vol's blocks dealt to the XCDs in runs of 64 (4096 queries) instead of contiguous
                         // eighths: r04c at cfg4, volume kernel 3.80 -> 3.50 ms, Mmg-like numbering 5.83 -> 4.14 ms
                         // (measurement build: PMMG_HIP_XCDRUN, 0 = eighths)
  // carry-over (pmmg_hip_keep / pmmg_hip_carry_over): kept[slot] holds the new
  // points and written rows of a host-mode call; an armed carry (carry_slot
  // >= 0) feeds the next host-mode set_background / set_solutions from it
  struct Kept {
    DevBuf xyz, met;
    std::vector<DevBuf> f;
    int np = 0, met_size = 0;
    std::vector<int> fsize;
    bool valid = false;
  };
  std::vector<Kept> kept;
  int last_host_np = 0, last_host_met = 0; // the last host-mode locate_interp (what pmmg_hip_keep keeps)
  std::vector<int> last_host_fsize;
  int carry_slot = -1, carry_np = 0;
  bool carry_bg = false;       // set_background took its vertices from the carry
  std::vector<int> carry_src;  // next vertex i+1 = kept point carry_src[i] (0: host row); empty: identity
  DevBuf carry_dsrc, carry_need, carry_ids, carry_cnt, carry_rows, carry_bc;
  int64_t bytes_up = 0; // host -> device bytes of host-mode calls (pmmg_hip_bytes_up)
  // pmmg_hip_locate_interp_groups: lanes[j] is lane j (same device and
  // options, created at the first groups call); lane 0 enqueues on this
  // context's own streams (no extra hardware queue) but has its own state, so
  // a groups call leaves this context's background and solutions as they were
  std::vector<pmmg_hip_ctx *> lanes;
  bool borrowed_streams = false; // a lane 0: stream / stream2 belong to its parent
  // the split of a group over the node's GPUs (pmmg_comm.hpp): an RCCL
  // communicator, owned (pmmg_hip_comm_init) or the caller's (attach)
  ncclComm_t comm = nullptr;
  bool comm_owned = false;
  int comm_rank = 0, comm_size = 0;
  DevBuf ag_send, ag_recv, ag_off, ag_chk; // (ag_chk: the all-gather's agreement, ag_agree)
  // PMMG_HIP_GROUP_LANES: most lanes of a groups call (r05k, 10 cfg2-size groups, 4 hardware queues: 4 / 5 /
  // 8 / 10 lanes 0.096 / 0.083 / 0.092 / 0.095 ms per group — 5 lanes take 2 groups each, 4 take 3, 3, 2, 2;
  // more hardware queues made it slower: 8 queues, 5 lanes 0.127; r04i: 1 / 2 lanes 0.165 / 0.125)
  // r06 (profiles/r06m, 3 rounds each, after a fresh start / after a large call in the process): 5 lanes of
  // 2 streams 0.090 / 0.106 ms per group, 4 x 2 0.079 / 0.091, 4 x 1 0.096 / 0.103, 5 x 1 0.096 / 0.085,
  // 3 x 1 0.081 / 0.082.  The hardware has 4 queues (GPU_MAX_HW_QUEUES): lane 0 on this context's two
  // streams plus two lanes of one stream each is 4 streams, one per queue whatever queues earlier streams of
  // the process left (a new stream takes the least used queue, ties broken in an order that changes from
  // process to process: with 10 streams two busy lanes shared a queue in some processes and not in others —
  // the r05 "slowdown after a large call")
  int group_lanes = 3;
  struct Pool *lane_pool = nullptr; // host threads enqueueing the other lanes' groups
  int lane_streams = 1; // a group lane's streams: 2 = its own surface stream, 1 = the surface branch on the
                        // main stream (measurement build: PMMG_HIP_LANE_STREAMS)
  int bdy_first = 0; // measurement build, PMMG_HIP_BDYFIRST=1: the volume kernel waits for the surface branch
  int bdy_after = 0; // measurement build, PMMG_HIP_BDYAFTER=1: k_bdy waits for the volume kernel (large calls)
  int vol_wait_seed = 0; // measurement build, PMMG_HIP_VOLWAIT=1: the volume kernel waits for the surface seeds
  int lane0 = 1; // lane 0 enqueues on this context's streams (measurement build: PMMG_HIP_LANE0=0 gives it
                 // streams of its own)
  // the volume stage split into a walk kernel that writes located records and an interpolation kernel
  // (r06), measured and not the default: at cfg4 the fused kernel's volume stage 3.30-3.35 ms,
  // split 3.60-3.66 (arrays) / 3.52 (packed records, one pass), chunked with the interpolation on its own stream
  // beside the next walk chunk 3.62-3.77 (profiles/r06a-r06c): the walk alone takes 1.91 ms and the
  // interpolation alone 1.90-1.99, whose sum the fused kernel beats by overlapping them across its waves, and
  // the located records add 1.9 GB of traffic.  PMMG_HIP_VOLSPLIT: 1 split (every call), 0 fused (default);
  // -1 split for calls of >= kSmallGroup queries
  int vol_split = 0;
  DevBuf locv, locp; // the split stage's located records (LocBuf): vertex ids, coordinates
  // the split stage in chunks: walk chunk j on the main stream, its interpolation on stream_i after the
  // chunk's event, so that interpolation j runs beside walk j + 1 (PMMG_HIP_VOLCHUNKS, 1..kMaxVolChunks)
  static constexpr int kMaxVolChunks = 16;
  int vol_chunks = 4;
  hipStream_t stream_i = nullptr;
  hipEvent_t ev_chunk[2][kMaxVolChunks] = {};
  hipEvent_t ev_interp = nullptr;
  int ixcd_run = -1; // measurement build, PMMG_HIP_IXCDRUN: the interpolation kernel's XCD run (-1: xcd_run)
  int null_sync = 0;   // measurement build, PMMG_HIP_NULLSYNC=1: small reads through the null stream (ctx_d2h)
  int eager_lanes = 0; // measurement build, PMMG_HIP_EAGERLANES=1: the group lanes created with the context
  int wave_time = 0;   // measurement build, PMMG_HIP_WAVETIME=1: k_bdy's per-wave wall-clock records, appended
                       // to the file PMMG_HIP_WAVETIME_OUT at each call's statistics
  DevBuf wt;
  size_t wt_n = 0;
  int filter_steps = 64; // step cap of the fp32 filter walk (then the exact fp64 walk continues from where it
                         // stopped: a query the filter misjudges hands over early instead of cycling through a
                         // 4-entry history for up to maxstep steps); test-only PMMG_HIP_FILTER_STEPS=0 sends every
                         // volume query to the exact walk
};

static void set_err(pmmg_hip_ctx *c, const char *fmt, ...) {
  if (!c) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(c->err, sizeof(c->err), fmt, ap);
  va_end(ap);
  fprintf(stderr, "[parmmg_hip] %s\n", c->err);
}

#define HIPCK(ctx, expr)                                                                             \
  do {                                                                                               \
    hipError_t e_ = (expr);                                                                          \
    if (e_ != hipSuccess) {                                                                          \
      set_err((ctx), "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);   \
      return 0;                                                                                      \
    }                                                                                                \
  } while (0)

// Device -> host reads of a context's small state on its own stream (r06):
// a synchronous hipMemcpy goes through the device's null stream, whose queue
// user — created at the first such copy — shifted the hardware queues the
// group lanes' streams were later given (the groups call
// 25 % slower after any earlier call in the process; tools/groups_probe.py,
// profiles/r06f).  PMMG_HIP_NULLSYNC=1 (measurement build): the null stream again.
static hipError_t ctx_d2h(pmmg_hip_ctx *c, void *dst, const void *src, size_t n) {
  if (c->null_sync) return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
  hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream);
  return e != hipSuccess ? e : hipStreamSynchronize(c->stream);
}

static int ensure(pmmg_hip_ctx *c, DevBuf &b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return 1;
  if (b.p) {
    HIPCK(c, hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  HIPCK(c, hipMalloc(&b.p, bytes));
  b.cap = bytes;
  return 1;
}

// the host-mode copy stream, created at the first host-mode upload (a
// device-mode context, and every group lane, keeps to two streams: the
// process has few hardware queues, GPU_MAX_HW_QUEUES = 4 by default, and
// streams beyond them share one)
static int copy_stream(pmmg_hip_ctx *c) {
  if (!c->cstream) HIPCK(c, hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
  return 1;
}

static void release(DevBuf &b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
}

// ---------------------------------------------------------------- host-mode transfers
//
// PMMG_HIP_HOST arrays are pageable host memory (the MMG5 arrays a shim
// hands over).  A DMA from pageable memory runs at ~35 GB/s (the runtime
// stages it through its own small pinned buffers one at a time); here the
// context owns two 32 MiB pinned buffers: host threads copy chunk j into one
// while the DMA engine moves chunk j-1 out of the other (and the reverse for
// downloads, where the host side also scatters only the rows the step wrote).

struct Pool { // fixed host threads running [begin, end) slices of one job at a time
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done;
  std::function<void(size_t, size_t)> fn;
  size_t n = 0, parts = 0, next = 0, left = 0;
  unsigned long long gen = 0;
  bool stop = false;
  explicit Pool(int nthreads) {
    for (int t = 0; t < nthreads; t++) th.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  bool take(size_t &b, size_t &e) { // under mu
    if (next >= parts) return false;
    const size_t p = next++;
    b = n * p / parts;
    e = n * (p + 1) / parts;
    return true;
  }
  void loop() {
    unsigned long long seen = 0;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || gen != seen; });
      if (stop) return;
      seen = gen;
      size_t b, e;
      while (take(b, e)) {
        lk.unlock();
        fn(b, e);
        lk.lock();
        if (--left == 0) done.notify_all();
      }
    }
  }
  void run(size_t count, size_t nparts, std::function<void(size_t, size_t)> f) {
    if (nparts <= 1 || th.empty()) {
      f(0, count);
      return;
    }
    std::unique_lock<std::mutex> lk(mu);
    fn = std::move(f);
    n = count;
    parts = nparts;
    next = 0;
    left = nparts;
    gen++;
    cv.notify_all();
    size_t b, e;
    while (take(b, e)) {
      lk.unlock();
      fn(b, e);
      lk.lock();
      left--;
    }
    done.wait(lk, [&] { return left == 0; });
  }
};

static int env_int(const char *name, int def);

constexpr size_t kStageBytes = 32u << 20;
constexpr size_t kStageMin = 4u << 20; // smaller copies go straight through the runtime
constexpr unsigned long long kSentinel = 0x7FF4A5A5A5A5A5A5ULL; // a signalling NaN no arithmetic produces

// device -> pinned host copies by a kernel (the GPU's PCIe writes into the
// mapped staging buffer; used for every host-mode download)
__global__ __launch_bounds__(kBlock) void k_copy16(const ntd2 *src, ntd2 *dst, long long n) {
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < n; j += (long long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + j), dst + j);
}
__global__ __launch_bounds__(kBlock) void k_copy1(const char *src, char *dst, long long n) {
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < n; j += (long long)gridDim.x * blockDim.x)
    dst[j] = src[j];
}

static int stage_ready(pmmg_hip_ctx *c) {
  if (c->stage[0]) return 1;
  for (int b = 0; b < 2; b++) {
    HIPCK(c, hipHostMalloc(&c->stage[b], kStageBytes, hipHostMallocDefault));
    HIPCK(c, hipHostGetDevicePointer(&c->stage_dev[b], c->stage[b], 0));
    HIPCK(c, hipEventCreateWithFlags(&c->stage_ev[b], hipEventDisableTiming));
  }
  if (!c->pool) {
    // helper threads for the staging copies: 15 (a one-GPU lease of the pool
    // gives 16 CPUs; hardware_concurrency shows the whole machine), fewer on
    // a smaller host, PMMG_HIP_HOST_THREADS to override
    const int hw = (int)std::thread::hardware_concurrency();
    c->pool = new Pool(env_int("PMMG_HIP_HOST_THREADS", hw > 16 ? 16 : (hw > 1 ? hw : 1)) - 1);
  }
  return 1;
}

static void par_copy(pmmg_hip_ctx *c, void *dst, const void *src, size_t n) {
  const size_t parts = n >= (8u << 20) ? c->pool->th.size() + 1 : 1;
  c->pool->run(n, parts, [&](size_t b, size_t e) { memcpy((char *)dst + b, (const char *)src + b, e - b); });
}

// host -> device, queued on the context stream; the host buffer may be
// reused as soon as the call returns
static int h2d(pmmg_hip_ctx *c, void *dst, const void *src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return 1;
  c->bytes_up += (int64_t)bytes;
  if (bytes < kStageMin) {
    HIPCK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return 1;
  }
  if (!stage_ready(c)) return 0;
  for (size_t off = 0; off < bytes;) {
    const int b = c->stage_i;
    c->stage_i ^= 1;
    const size_t n = bytes - off < kStageBytes ? bytes - off : kStageBytes;
    HIPCK(c, hipEventSynchronize(c->stage_ev[b])); // the buffer's previous DMA is done
    par_copy(c, c->stage[b], (const char *)src + off, n);
    HIPCK(c, hipMemcpyAsync((char *)dst + off, c->stage[b], n, hipMemcpyHostToDevice, s));
    HIPCK(c, hipEventRecord(c->stage_ev[b], s));
    off += n;
  }
  return 1;
}

// device -> host of nrows rows of `row` bytes; keep(r, bytes) selects the rows
// copied into dst (AllRows: every row, one plain copy).  Synchronous.
struct AllRows {
  bool operator()(size_t, const char *) const { return true; }
};
static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class Keep>
static int d2h_rows(pmmg_hip_ctx *c, void *dst, const void *src, size_t nrows, size_t row, const Keep &keep) {
  const size_t bytes = nrows * row;
  if (bytes == 0) return 1;
  if (!stage_ready(c)) return 0;
  double t_wait = 0.0;
  const double t_start = now_s();
  const size_t per = kStageBytes / row; // rows per chunk
  const size_t nch = (nrows + per - 1) / per;
  auto issue = [&](size_t j) -> int {
    const int b = (int)(j & 1);
    const size_t r0 = j * per, n = (nrows - r0 < per ? nrows - r0 : per) * row;
    // the GPU writes the chunk into the mapped pinned buffer: its PCIe writes
    // reach ~2x the rate of the DMA engine's device->host copies (r02m: 48-byte
    // row arrays 36 -> 20-24 ms per GB; the host-side scatter now bounds it)
    const char *from = (const char *)src + r0 * row;
    if (((uintptr_t)from & 15) == 0 && (n & 15) == 0) {
      hipLaunchKernelGGL(k_copy16, dim3(1024), dim3(kBlock), 0, c->stream, (const ntd2 *)from, (ntd2 *)c->stage_dev[b],
                         (long long)(n / 16));
    } else {
      hipLaunchKernelGGL(k_copy1, dim3(1024), dim3(kBlock), 0, c->stream, from, (char *)c->stage_dev[b], (long long)n);
    }
    HIPCK(c, hipGetLastError());
    HIPCK(c, hipEventRecord(c->stage_ev[b], c->stream));
    return 1;
  };
  if (!issue(0)) return 0;
  for (size_t j = 0; j < nch; j++) {
    const int b = (int)(j & 1);
    const double t0 = now_s();
    HIPCK(c, hipEventSynchronize(c->stage_ev[b]));
    const double t1 = now_s();
    t_wait += t1 - t0;
    if (j + 1 < nch && !issue(j + 1)) return 0; // the next chunk moves while this one is scattered
    const size_t r0 = j * per, nr = nrows - r0 < per ? nrows - r0 : per;
    const char *sb = (const char *)c->stage[b];
    char *db = (char *)dst + r0 * row;
    if constexpr (std::is_same<Keep, AllRows>::value) {
      par_copy(c, db, sb, nr * row);
    } else {
      // runs of consecutive kept rows go out as one memcpy each (nearly every
      // row is kept in a transfer: one copy per slice instead of one per row)
      c->pool->run(nr, nr >= 65536 ? c->pool->th.size() + 1 : 1, [&](size_t a, size_t e) {
        size_t r = a;
        while (r < e) {
          while (r < e && !keep(r0 + r, sb + r * row)) r++;
          const size_t s0 = r;
          while (r < e && keep(r0 + r, sb + r * row)) r++;
          if (r > s0) memcpy(db + s0 * row, sb + s0 * row, (r - s0) * row);
        }
      });
    }
  }
  if (c->verbose)
    fprintf(stderr, "[parmmg_hip] d2h %zu rows x %zu B: %.2f ms DMA wait, %.2f ms in total\n", nrows, row,
            1e3 * t_wait, 1e3 * (now_s() - t_start));
  return 1;
}

static int upload(pmmg_hip_ctx *c, DevBuf &b, const void *src, size_t bytes, hipStream_t s = nullptr) {
  if (!ensure(c, b, bytes)) return 0;
  return h2d(c, b.p, src, bytes, s ? s : c->stream);
}

// a background whose snapshot failed is dropped: its tet8 adjacency or
// boundary trias may be partly written, so no later call may walk it (the
// 'no background set' guard then fails them until set_background succeeds)
static void invalidate_bg(pmmg_hip_ctx *c) {
  c->bg.ne = c->bg.nt = c->bg.np = 0;
  c->bg.tetv = c->bg.adja = nullptr;
  c->bg.triv = c->bg.adjt = nullptr;
  c->bg.xyz = nullptr;
}

// wait for a deferred device snapshot (host-mode set_background); 0 if it failed
static int snap_join(pmmg_hip_ctx *c) {
  if (c->snap.joinable()) c->snap.join();
  if (!c->snap_ok) {
    c->snap_ok = 1; // reported once, by the call that joined it
    invalidate_bg(c);
    return 0;
  }
  return 1;
}

// 16-byte streaming stores (a from hipMalloc: 16-byte aligned); the odd last
// element by the first thread.  (r05: 8-byte stores refilled cfg4's 101 MB
// seed grid in 43 us, ~2.3 TB/s)
typedef unsigned long long ntu2 __attribute__((ext_vector_type(2)));
__global__ void k_fill64(unsigned long long *a, long long n, unsigned long long v) {
  const ntu2 vv = {v, v};
  const long long n2 = n >> 1;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < n2; j += (long long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(vv, reinterpret_cast<ntu2 *>(a) + j);
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) a[n - 1] = v;
}
__global__ void k_fill32(int *a, long long n, int v) {
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < n; j += (long long)gridDim.x * blockDim.x)
    a[j] = v;
}
// seed grids of at least this many cells are refilled at the end of the call
// that used them; smaller ones (a small group's chain of launches is its
// cost) are cleared by k_reset
constexpr long long kRefillCells = 1LL << 20;

static int env_int(const char *name, int def) { // positive values only
  const char *e = getenv(name);
  if (e && atoi(e) > 0) return atoi(e);
  return def;
}
// switches whose 0 (or -1) is a setting of its own (env_int reads 0 as unset: up to r06zm the
// PMMG_HIP_HOSTORDER=0, FUSECONT=0, SRFSOLO=0, LANE0=0, STREAM3=0 and IXCDRUN=0 variants ran the default)
static int env_int_any(const char *name, int def) {
  const char *e = getenv(name);
  if (!e || !*e) return def;
  char *end = nullptr;
  const long v = strtol(e, &end, 10);
  return (end && *end == 0) ? (int)v : def;
}

extern "C" {

int pmmg_hip_abi_version(void) { return PMMG_HIP_ABI_VERSION; }
int64_t pmmg_hip_stats_size(void) { return (int64_t)sizeof(pmmg_hip_stats); }

int pmmg_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// share != NULL: a group lane that enqueues on share's two streams (its
// own buffers, events and state; the streams are not destroyed with it)
static pmmg_hip_ctx *create_ctx(int device, int options, bool srf_prio, pmmg_hip_ctx *share = nullptr) {
  int n = pmmg_hip_device_count();
  if (n <= 0 || device < 0 || device >= n) {
    fprintf(stderr, "[parmmg_hip] no HIP device %d (visible: %d)\n", device, n);
    return nullptr;
  }
  pmmg_hip_ctx *c = new pmmg_hip_ctx();
  c->device = device;
  c->options = options;
#ifdef PMMG_HIP_MEASURE
  if (const char *e = getenv("PMMG_HIP_SRFPRIO"))
    if (*e == '1') c->srf_prio = srf_prio;
#else
  (void)srf_prio;
#endif
  if (share) {
    c->stream = share->stream;
    c->stream2 = share->stream2;
    c->borrowed_streams = true;
  }
  if (hipSetDevice(device) != hipSuccess ||
      (!share && (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
                  hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess))) {
    fprintf(stderr, "[parmmg_hip] cannot initialise device %d\n", device);
    delete c;
    return nullptr;
  }
  {
    // measurement build, PMMG_HIP_EVFLAGS: 1 = the call's events without the system-scope fence, 2 = with a
    // device-scope release; the order decision's EV_FRAME (read by the host) and EV_END keep the default
    int evf = 0;
#ifdef PMMG_HIP_MEASURE
    evf = env_int("PMMG_HIP_EVFLAGS", 0);
#endif
    const unsigned fl = evf == 1 ? hipEventDisableSystemFence : (evf == 2 ? hipEventReleaseToDevice : 0u);
    for (int i = 0; i < EV_COUNT; i++)
      (void)hipEventCreateWithFlags(&c->ev[i], (i == EV_FRAME || i == EV_END) ? hipEventDefault : fl);
  }
  // documented options, each clamped to its valid range
  c->tpc = std::min(4096, env_int("PMMG_HIP_TPC", c->tpc));
  c->srf_mult = std::min(4096, env_int("PMMG_HIP_SRFMULT", c->srf_mult));
  c->bin_bits = std::min(7, env_int("PMMG_HIP_BINBITS", c->bin_bits));
  c->verbose = env_int("PMMG_HIP_VERBOSE", 0);
  c->maxstep = env_int("PMMG_HIP_MAXSTEP", c->maxstep);
  c->group_lanes = std::min(16, env_int("PMMG_HIP_GROUP_LANES", c->group_lanes));
  // test-only path selection (tests/test_gpu_hits.py, tests/test_gpu_parity.py)
  c->fanmax = env_int("PMMG_HIP_FANMAX", c->fanmax);
  c->srf_g = std::min(1024, env_int("PMMG_HIP_SRFG", 0));
  c->pack_passes = std::max(0, std::min(2, env_int("PMMG_HIP_PACKPASS", c->pack_passes))); // packed: gather passes
  if (const char *e = getenv("PMMG_HIP_VOLSPLIT"))
    if (*e == '0' || *e == '1') c->vol_split = *e - '0';
  c->vol_chunks = std::max(1, std::min((int)pmmg_hip_ctx::kMaxVolChunks, env_int("PMMG_HIP_VOLCHUNKS", c->vol_chunks)));
  c->bg.fanmax = c->fanmax; // every kernel's Bg copy carries it
  c->filter_steps = c->filter_steps < c->maxstep ? c->filter_steps : c->maxstep;
  if (const char *e = getenv("PMMG_HIP_FILTER_STEPS"))
    if (*e && atoi(e) >= 0) c->filter_steps = atoi(e);
#ifdef PMMG_HIP_MEASURE
  // A/B switches of the measurement build (libpmmg_hip_measure.so, tools/)
  c->seed_lanes = std::min(4, env_int("PMMG_HIP_SEEDLANES", c->seed_lanes));
  c->seed_v0 = (env_int("PMMG_HIP_SEEDV0", 0) == 1 ? 1 : 0) | (env_int("PMMG_HIP_SEEDNOATOM", 0) == 1 ? 2 : 0);
  c->bbox_stride = env_int("PMMG_HIP_BBOX", c->bbox_stride);
  c->hist_stride = env_int("PMMG_HIP_HIST", c->hist_stride);
  c->bdy_dyn = (env_int("PMMG_HIP_BDYDYN", 2) == 1 ? 1 : 0) | (env_int("PMMG_HIP_BDYNOINTERP", 0) == 1 ? 2 : 0);
  c->bdy_bpx = env_int("PMMG_HIP_BDYBPX", c->bdy_bpx);
  c->bdy_wave = env_int("PMMG_HIP_BDYWAVE", c->bdy_wave);
  c->host_order = env_int_any("PMMG_HIP_HOSTORDER", c->host_order);
  c->fuse_cont = env_int_any("PMMG_HIP_FUSECONT", c->fuse_cont);
  c->quant_side = env_int("PMMG_HIP_QUANTSIDE", c->quant_side);
  c->bin_qs = env_int("PMMG_HIP_BINQS", 2) == 1;
  c->brick = env_int("PMMG_HIP_BRICK", 0);
  c->srf_solo = env_int_any("PMMG_HIP_SRFSOLO", -1);
  c->set_order = env_int("PMMG_HIP_SETORDER", 0);
  if (const char *e = getenv("PMMG_HIP_XCDRUN"))
    if (*e && atoi(e) >= 0) c->xcd_run = atoi(e);
  c->pad = env_int("PMMG_HIP_PAD", 0);
  c->ixcd_run = env_int_any("PMMG_HIP_IXCDRUN", -1);
  c->null_sync = env_int("PMMG_HIP_NULLSYNC", 0);
  c->eager_lanes = env_int("PMMG_HIP_EAGERLANES", 0);
  c->wave_time = env_int("PMMG_HIP_WAVETIME", 0);
  c->lane_streams = std::max(1, std::min(3, env_int("PMMG_HIP_LANE_STREAMS", c->lane_streams)));
  c->lane0 = env_int_any("PMMG_HIP_LANE0", 1) ? 1 : 0;
  c->bdy_first = env_int("PMMG_HIP_BDYFIRST", 0);
  c->bdy_after = env_int("PMMG_HIP_BDYAFTER", 0);
  c->vol_wait_seed = env_int("PMMG_HIP_VOLWAIT", 0);
  c->no_fb = env_int("PMMG_HIP_NOFB", 0);
  c->stream3_mode = env_int_any("PMMG_HIP_STREAM3", c->stream3_mode);
  if (c->stream3_mode == 2 && hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking) != hipSuccess)
    c->stream3 = nullptr; // the exhaustive kernels not launched (a launch's price; wrong results
                                           // wherever a query needs them)
#endif
  return c;
}

static pmmg_hip_ctx *group_lane(pmmg_hip_ctx *c, int j);

pmmg_hip_ctx *pmmg_hip_create(int device, int options) {
  pmmg_hip_ctx *c = create_ctx(device, options, true);
  if (c && c->eager_lanes)
    for (int j = 0; j < c->group_lanes; j++) (void)group_lane(c, j);
  return c;
}

void pmmg_hip_destroy(pmmg_hip_ctx *c) {
  if (!c) return;
  delete c->lane_pool;
  for (pmmg_hip_ctx *l : c->lanes) pmmg_hip_destroy(l);
  (void)hipSetDevice(c->device);
  (void)snap_join(c);
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->stream2);
  if (c->stream2_hi) (void)hipStreamSynchronize(c->stream2_hi);
  if (c->stream3) (void)hipStreamSynchronize(c->stream3);
  if (c->stream_f) (void)hipStreamSynchronize(c->stream_f);
  if (c->cstream) (void)hipStreamSynchronize(c->cstream);
  if (c->stream_i) {
    (void)hipStreamSynchronize(c->stream_i);
    (void)hipStreamDestroy(c->stream_i);
  }
  for (auto &row : c->ev_chunk)
    for (hipEvent_t &e : row)
      if (e) (void)hipEventDestroy(e);
  if (c->ev_interp) (void)hipEventDestroy(c->ev_interp);
  DevBuf *bufs[] = {&c->o_xyz, &c->o_tetv, &c->o_adja, &c->o_triv, &c->o_adjt, &c->o_met, &c->o_rec, &c->frame,
                    &c->stats, &c->grid, &c->sgrid, &c->order_v, &c->cohd,
                    &c->order_b, &c->cont, &c->xq, &c->qs, &c->axh, &c->bkeys, &c->bkeys2, &c->bvals, &c->bvals2, &c->rs_hist, &c->rs_csum, &c->oflag, &c->cls_cnt, &c->qmin, &c->fb_vol, &c->fb_bdy,
                    &c->best, &c->nac, &c->cres, &c->bbest, &c->bnac, &c->bcres, &c->fbp_vol, &c->fbp_bdy, &c->fbg_vol_c,
                    &c->fbg_vol_u, &c->fbg_vol_i, &c->fbg_bdy_c, &c->fbg_bdy_u, &c->fbg_bdy_i, &c->h_xyz,
                    &c->h_cls, &c->h_met, &c->h_elem, &c->h_hit, &c->brk_k, &c->brk_k2, &c->brk_v, &c->brk_v2,
                    &c->brk_vinv, &c->brk_tinv, &c->brk_xq, &c->brk_xyz, &c->brk_sol, &c->brk_rec, &c->brk_tmp,
                    &c->locv, &c->locp, &c->wt};
  for (DevBuf *b : bufs) release(*b);
  for (auto &b : c->o_f) release(b);
  for (auto &b : c->h_f) release(b);
  for (int i = 0; i < EV_COUNT; i++)
    if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
  for (int b = 0; b < 2; b++) {
    if (c->stage[b]) (void)hipHostFree(c->stage[b]);
    if (c->stage_ev[b]) (void)hipEventDestroy(c->stage_ev[b]);
  }
  delete c->pool;
  release(c->o_tet4);
  pmmg_snap_cache_free(&c->snap_cache);
  for (auto &k : c->kept) {
    release(k.xyz);
    release(k.met);
    for (auto &b : k.f) release(b);
  }
  DevBuf *cb[] = {&c->carry_dsrc, &c->carry_need, &c->carry_ids, &c->carry_cnt, &c->carry_rows, &c->carry_bc,
                  &c->ag_send, &c->ag_recv, &c->ag_off, &c->ag_chk};
  for (DevBuf *b : cb) release(*b);
  if (c->comm && c->comm_owned && rccl().ok) (void)rccl().commDestroy(c->comm);
  if (!c->borrowed_streams) {
    if (c->stream2 && c->stream2 != c->stream) (void)hipStreamDestroy(c->stream2);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  }
  if (c->stream2_hi) (void)hipStreamDestroy(c->stream2_hi);
  if (c->stream3) (void)hipStreamDestroy(c->stream3);
  if (c->stream_f) (void)hipStreamDestroy(c->stream_f);
  if (c->flag_host) (void)hipHostFree(c->flag_host);
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  delete c;
}

const char *pmmg_hip_last_error(pmmg_hip_ctx *c) { return c ? c->err : "null context"; }

// ---------------------------------------------------------------- carry-over
//
// ParMmg's next iteration takes the adapted group as its old group
// (src/libparmmg1.c:653 -> PMMG_update_oldGrps, src/grpsplit_pmmg.c:1224-1248):
// its vertices are the new points the transfer step just located and its
// solutions the rows the step just wrote, both still in HBM after a
// host-mode call.  pmmg_hip_keep keeps them (the staging buffers are swapped
// into a slot, no copy); pmmg_hip_carry_over arms the next host-mode
// set_background / set_solutions to take from the slot every row it holds —
// vertex i + 1 of the new background is kept point src[i] — and to upload only
// the rest: vertices not in the slot (src[i] == 0, e.g. moved in by load
// balancing) and rows the step did not write (skipped points, whose values
// the caller copies on the host, and MMG5_invmat failures), found on the
// device by the output sentinel.

static int blocks_for(long long n, int cap);

// to[i] = from[src[i] - 1] (row doubles; src NULL: the identity, to NULL: no
// copy); need[i] = 1 where the row must come from the host: src[i] == 0, or
// (check) the kept row is the unwritten sentinel
__global__ void k_carry_gather(const double *from, int row, const int *src, long long np, double *to, uint8_t *need,
                               int check) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < np; i += (long long)gridDim.x * blockDim.x) {
    const long long s = src ? (long long)src[i] : i + 1;
    bool miss = s <= 0;
    if (!miss) {
      const double *f = from + (size_t)row * (size_t)(s - 1);
      miss = check && (unsigned long long)__double_as_longlong(f[0]) == kSentinel;
      if (!miss && to)
        for (int j = 0; j < row; j++) to[(size_t)row * (size_t)i + j] = f[j];
    }
    if (miss && need) need[i] = 1;
  }
}

// to[ids[k] - 1] = rows[k] (row doubles), k < *n
__global__ void k_scatter_rows(const double *rows, const int *ids, const int *n, int row, double *to) {
  for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < *n; k += (long long)gridDim.x * blockDim.x)
    for (int j = 0; j < row; j++) to[(size_t)row * (size_t)(ids[k] - 1) + j] = rows[(size_t)row * (size_t)k + j];
}

// host rows ids (1-based) of `host` uploaded and scattered into dst
static int carry_host_rows(pmmg_hip_ctx *c, const std::vector<int> &ids, const double *host, int row, double *dst) {
  if (ids.empty()) return 1;
  std::vector<double> rows((size_t)row * ids.size());
  for (size_t k = 0; k < ids.size(); k++)
    memcpy(&rows[(size_t)row * k], host + (size_t)row * (size_t)(ids[k] - 1), sizeof(double) * row);
  const int n = (int)ids.size();
  if (!upload(c, c->carry_rows, rows.data(), sizeof(double) * rows.size()) ||
      !upload(c, c->carry_ids, ids.data(), sizeof(int) * ids.size()) || !upload(c, c->carry_cnt, &n, sizeof(int)))
    return 0;
  hipLaunchKernelGGL(k_scatter_rows, dim3(blocks_for(n, 4096)), dim3(kBlock), 0, c->stream,
                     (const double *)c->carry_rows.p, (const int *)c->carry_ids.p, (const int *)c->carry_cnt.p, row,
                     dst);
  HIPCK(c, hipGetLastError());
  return 1;
}

static void carry_disarm(pmmg_hip_ctx *c) {
  c->carry_slot = -1;
  c->carry_bg = false;
  c->carry_src.clear();
}

// set_background, host mode, carry armed: the vertices from the slot
static int carry_vertices(pmmg_hip_ctx *c, int np, const double *xyz) {
  pmmg_hip_ctx::Kept &k = c->kept[c->carry_slot];
  if (np != c->carry_np || c->carry_bg) {
    set_err(c, "set_background: the armed carry-over is for %d vertices (got %d)%s", c->carry_np, np,
            c->carry_bg ? " and was taken already" : "");
    carry_disarm(c);
    return 0;
  }
  k.valid = false; // the slot is consumed by this carry, whatever happens next (a swapped-out
                   // buffer must never feed a later carry of the same slot)
  if (c->carry_src.empty()) {
    std::swap(c->o_xyz, k.xyz); // every row is a kept point, in order
  } else {
    if (!ensure(c, c->o_xyz, sizeof(double) * 3 * (size_t)np) ||
        !upload(c, c->carry_dsrc, c->carry_src.data(), sizeof(int) * (size_t)np)) {
      carry_disarm(c);
      return 0;
    }
    hipLaunchKernelGGL(k_carry_gather, dim3(blocks_for(np, 4096)), dim3(kBlock), 0, c->stream,
                       (const double *)k.xyz.p, 3, (const int *)c->carry_dsrc.p, (long long)np, (double *)c->o_xyz.p,
                       (uint8_t *)nullptr, 0);
    std::vector<int> ids;
    for (int i = 0; i < np; i++)
      if (c->carry_src[i] == 0) ids.push_back(i + 1);
    if (!carry_host_rows(c, ids, xyz, 3, (double *)c->o_xyz.p)) {
      carry_disarm(c);
      return 0;
    }
  }
  c->carry_bg = true;
  return 1;
}

// set_solutions, host mode, carry armed: the metric and the fields whose
// sizes match the kept ones from the slot, their missing rows from the host
static int carry_solutions_body(pmmg_hip_ctx *c, int met_size, const double *met, int nfield, const int *field_size,
                                const double *const *fields);

// every way out of an armed set_solutions disarms the carry
static int carry_solutions(pmmg_hip_ctx *c, int met_size, const double *met, int nfield, const int *field_size,
                           const double *const *fields) {
  const int ok = carry_solutions_body(c, met_size, met, nfield, field_size, fields);
  carry_disarm(c);
  return ok;
}

static int carry_solutions_body(pmmg_hip_ctx *c, int met_size, const double *met, int nfield, const int *field_size,
                                const double *const *fields) {
  pmmg_hip_ctx::Kept &k = c->kept[c->carry_slot];
  const int np = c->carry_np;
  const bool ident = c->carry_src.empty();
  hipStream_t s = c->stream;
  if (!c->carry_bg || np != c->bg.np) {
    set_err(c, "set_solutions: the armed carry-over needs set_background with its %d vertices first", np);
    carry_disarm(c);
    return 0;
  }
  const long long ncls = np / kScanChunk + 1;
  if (!ensure(c, c->carry_need, (size_t)np) || !ensure(c, c->carry_ids, sizeof(int) * (size_t)np) ||
      !ensure(c, c->carry_cnt, sizeof(int)) || !ensure(c, c->carry_bc, sizeof(int) * (size_t)ncls))
    return 0;
  HIPCK(c, hipMemsetAsync(c->carry_need.p, 0, (size_t)np, s));
  struct Arr { DevBuf *dst; const double *host; int row; };
  std::vector<Arr> carried;
  auto take = [&](DevBuf &dst, DevBuf &from, const double *host, int row) -> int {
    if (ident) {
      std::swap(dst, from);
      hipLaunchKernelGGL(k_carry_gather, dim3(blocks_for(np, 4096)), dim3(kBlock), 0, s, (const double *)dst.p, row,
                         (const int *)nullptr, (long long)np, (double *)nullptr, (uint8_t *)c->carry_need.p, 1);
    } else {
      if (!ensure(c, dst, sizeof(double) * row * (size_t)np)) return 0;
      hipLaunchKernelGGL(k_carry_gather, dim3(blocks_for(np, 4096)), dim3(kBlock), 0, s, (const double *)from.p, row,
                         (const int *)c->carry_dsrc.p, (long long)np, (double *)dst.p, (uint8_t *)c->carry_need.p, 1);
    }
    HIPCK(c, hipGetLastError());
    carried.push_back(Arr{&dst, host, row});
    return 1;
  };
  // what is not carried goes up whole
  if (met_size) {
    if (k.met_size == met_size && k.met.p) {
      if (!take(c->o_met, k.met, met, met_size)) return 0;
    } else if (!copy_stream(c) || !upload(c, c->o_met, met, sizeof(double) * met_size * (size_t)np, c->cstream)) {
      return 0;
    }
    c->met = (const double *)c->o_met.p;
  }
  c->o_f.resize(nfield);
  for (int j = 0; j < nfield; j++) {
    if (j < (int)k.f.size() && k.fsize[j] == field_size[j] && k.f[j].p) {
      if (!take(c->o_f[j], k.f[j], fields[j], field_size[j])) return 0;
    } else if (!copy_stream(c) ||
               !upload(c, c->o_f[j], fields[j], sizeof(double) * field_size[j] * (size_t)np, c->cstream)) {
      return 0;
    }
    c->fin[j] = (const double *)c->o_f[j].p;
  }
  if (!carried.empty()) {
    // the rows to fetch from the host: one list for every carried array
    const uint8_t *need = (const uint8_t *)c->carry_need.p;
    int *bc = (int *)c->carry_bc.p;
    hipLaunchKernelGGL(k_cls_count, dim3((unsigned)ncls), dim3(kBlock), 0, s, need, (long long)np, 1, bc,
                       (const int *)nullptr, 0);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, s, bc, (int)ncls, (int *)c->carry_cnt.p,
                       (const int *)nullptr, 0);
    hipLaunchKernelGGL(k_cls_scatter, dim3((unsigned)ncls), dim3(kBlock), 0, s, need, (long long)np, 1,
                       (const int *)bc, (int *)c->carry_ids.p, (const int *)nullptr, 0);
    HIPCK(c, hipGetLastError());
    int n = 0;
    HIPCK(c, hipMemcpyAsync(&n, c->carry_cnt.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCK(c, hipStreamSynchronize(s));
    std::vector<int> ids((size_t)n);
    if (n > 0) HIPCK(c, ctx_d2h(c, ids.data(), c->carry_ids.p, sizeof(int) * (size_t)n));
    for (const Arr &a : carried)
      if (!carry_host_rows(c, ids, a.host, a.row, (double *)a.dst->p)) return 0;
  }
  if (c->cstream) HIPCK(c, hipStreamSynchronize(c->cstream));
  HIPCK(c, hipStreamSynchronize(s));
  k.valid = false; // its buffers now back the background (or were swapped out)
  carry_disarm(c);
  return 1;
}

// shared body of the two background entry points: tet8 != NULL selects the
// packed {v[4], adja[4]} records, else the separate tetv / adja arrays.
// adja == NULL: the adjacency is built on the device (MMG3D_hashTetra's
// result, into owned tet8 records); triv == NULL with nt < 0: the boundary
// trias and their adjacency are built on the device (MMG5_chkBdryTria +
// MMG3D_hashTria for an old mesh without input trias); adjt == NULL with
// triv given: the tria adjacency is built on the device.
static int set_background_impl(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tetv, const int *adja,
                               const int *tet8, int nt, const int *triv, const int *adjt, double hausd, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  const bool packed = tet8 != nullptr;
  const bool build_bdy = nt < 0 && !triv;
  if (np <= 0 || ne <= 0 || !xyz || (!packed && !tetv) || (nt < 0 && triv) || (nt > 0 && !triv)) {
    set_err(c, "set_background: invalid arguments (np=%d ne=%d nt=%d)", np, ne, nt);
    return 0;
  }
  if (ne >= (1 << 29)) {
    set_err(c, "set_background: %d tetra exceed the 4*k+i adjacency encoding (2^29)", ne);
    return 0;
  }
  const bool dev = where == PMMG_HIP_DEVICE;
  if (dev) {
    const void *t0 = packed ? (const void *)tet8 : (const void *)tetv;
    if (((uintptr_t)t0 & 15) || (!packed && adja && ((uintptr_t)adja & 15))) {
      set_err(c, "set_background: device tetra arrays must be 16-byte aligned");
      return 0;
    }
  }
  c->bg.np = np;
  c->bg.ne = ne;
  c->bg.hausd = hausd;
  // vertices
  if (dev) {
    if (c->carry_slot >= 0) {
      set_err(c, "set_background: a carry-over is armed; it takes host-mode (PMMG_HIP_HOST) calls");
      carry_disarm(c);
      return 0;
    }
    c->bg.xyz = xyz;
  } else {
    if (c->carry_slot >= 0) {
      if (!carry_vertices(c, np, xyz)) return 0;
    } else if (!upload(c, c->o_xyz, xyz, sizeof(double) * 3 * (size_t)np)) {
      return 0;
    }
    c->bg.xyz = (const double *)c->o_xyz.p;
  }
  // tetra
  const int *d_tetv = nullptr; // input of the device adjacency
  if (packed) {
    if (dev) {
      c->bg.tetv = reinterpret_cast<const int4 *>(tet8);
    } else {
      if (!upload(c, c->o_tetv, tet8, sizeof(int) * 8 * (size_t)ne)) return 0;
      c->bg.tetv = (const int4 *)c->o_tetv.p;
    }
    c->bg.adja = c->bg.tetv + 1;
    c->bg.tstride = 2;
  } else if (adja) {
    if (dev) {
      c->bg.tetv = reinterpret_cast<const int4 *>(tetv);
      c->bg.adja = reinterpret_cast<const int4 *>(adja);
    } else {
      if (!upload(c, c->o_tetv, tetv, sizeof(int) * 4 * (size_t)ne)) return 0;
      if (!upload(c, c->o_adja, adja, sizeof(int) * 4 * (size_t)ne)) return 0;
      c->bg.tetv = (const int4 *)c->o_tetv.p;
      c->bg.adja = (const int4 *)c->o_adja.p;
    }
    c->bg.tstride = 1;
  } else { // device adjacency into owned tet8 records
    d_tetv = tetv;
    if (!dev) {
      if (!upload(c, c->o_tet4, tetv, sizeof(int) * 4 * (size_t)ne)) return 0;
      d_tetv = (const int *)c->o_tet4.p;
    }
    if (!ensure(c, c->o_tetv, sizeof(int) * 8 * (size_t)ne)) return 0;
    c->bg.tetv = (const int4 *)c->o_tetv.p;
    c->bg.adja = c->bg.tetv + 1;
    c->bg.tstride = 2;
  }
  // boundary trias handed over
  if (!build_bdy) {
    if (dev) {
      c->bg.triv = triv;
      c->bg.adjt = adjt;
    } else {
      if (!upload(c, c->o_triv, triv, sizeof(int) * 3 * (size_t)nt)) return 0;
      c->bg.triv = (const int *)c->o_triv.p;
      c->bg.adjt = nullptr;
      if (adjt) {
        if (!upload(c, c->o_adjt, adjt, sizeof(int) * 3 * (size_t)nt)) return 0;
        c->bg.adjt = (const int *)c->o_adjt.p;
      }
    }
    c->bg.nt = nt;
  }
  const bool tria_adj = !build_bdy && nt > 0 && !adjt;
  // the device snapshot (PMMG_create_oldGrp's arrays): adjacency, boundary
  // trias, tria adjacency, each on the context stream
  auto snapshot = [c, np, ne, d_tetv, build_bdy, tria_adj]() -> int {
    if (d_tetv && !pmmg_snap_adjacency(c->stream, np, ne, d_tetv, nullptr, (int *)c->o_tetv.p, &c->snap_cache, c->err,
                                     sizeof(c->err))) {
      fprintf(stderr, "[parmmg_hip] %s\n", c->err);
      return 0;
    }
    if (build_bdy) {
      const int *t0 = reinterpret_cast<const int *>(c->bg.tetv), *a0 = reinterpret_cast<const int *>(c->bg.adja);
      int cnt = 0, ntb = 0;
      char msg[256];
      pmmg_snap_boundary(c->stream, np, ne, t0, c->bg.tstride, a0, c->bg.tstride, nullptr, 0, &cnt, nullptr, nullptr,
                         &c->snap_cache, msg, sizeof(msg)); // counts (fails on capacity 0 when there are trias)
      if (!ensure(c, c->o_triv, sizeof(int) * 3 * (size_t)cnt) || !ensure(c, c->o_adjt, sizeof(int) * 3 * (size_t)cnt))
        return 0;
      if (!pmmg_snap_boundary(c->stream, np, ne, t0, c->bg.tstride, a0, c->bg.tstride, nullptr, cnt, &ntb,
                              (int *)c->o_triv.p, (int *)c->o_adjt.p, &c->snap_cache, c->err, sizeof(c->err))) {
        fprintf(stderr, "[parmmg_hip] %s\n", c->err);
        return 0;
      }
      c->bg.triv = (const int *)c->o_triv.p;
      c->bg.adjt = (const int *)c->o_adjt.p;
      c->bg.nt = ntb;
    }
    if (tria_adj) {
      if (!ensure(c, c->o_adjt, sizeof(int) * 3 * (size_t)c->bg.nt)) return 0;
      if (!pmmg_snap_tria_adjacency(c->stream, np, c->bg.nt, c->bg.triv, (int *)c->o_adjt.p, &c->snap_cache, c->err,
                                    sizeof(c->err))) {
        fprintf(stderr, "[parmmg_hip] %s\n", c->err);
        return 0;
      }
      c->bg.adjt = (const int *)c->o_adjt.p;
    }
    return 1;
  };
  if (!dev && (d_tetv || build_bdy || tria_adj)) {
    // host mode: the snapshot runs in a host thread (its kernels on the
    // context stream) while the caller goes on to set_solutions, whose
    // uploads use the copy stream; the next other call joins it
    c->snap_ok = 1;
    c->snap = std::thread([c, snapshot] {
      c->snap_ok = hipSetDevice(c->device) == hipSuccess ? snapshot() : 0;
    });
    return 1;
  }
  if (!snapshot()) {
    invalidate_bg(c);
    return 0;
  }
  if (!dev) HIPCK(c, hipStreamSynchronize(c->stream));
  return 1;
}

int pmmg_hip_set_background(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tetv, const int *adja,
                            int nt, const int *triv, const int *adjt, double hausd, int where) {
  if (c && !tetv) {
    set_err(c, "set_background: tetv is NULL");
    return 0;
  }
  return set_background_impl(c, np, xyz, ne, tetv, adja, nullptr, nt, triv, adjt, hausd, where);
}

int pmmg_hip_set_background_tet8(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tet8, int nt,
                                 const int *triv, const int *adjt, double hausd, int where) {
  if (c && !tet8) {
    set_err(c, "set_background_tet8: tet8 is NULL");
    return 0;
  }
  return set_background_impl(c, np, xyz, ne, nullptr, nullptr, tet8, nt, triv, adjt, hausd, where);
}

int pmmg_hip_set_solutions(pmmg_hip_ctx *c, int met_size, const double *met, int nfield, const int *field_size,
                           const double *const *fields, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (met_size != 0 && met_size != 1 && met_size != 6) {
    set_err(c, "set_solutions: metric size %d (expected 0, 1 or 6)", met_size);
    return 0;
  }
  if (nfield < 0 || nfield + (met_size ? 1 : 0) > kMaxSlot) {
    set_err(c, "set_solutions: %d fields exceed the %d-slot limit", nfield, kMaxSlot);
    return 0;
  }
  if (met_size && !met) {
    set_err(c, "set_solutions: metric pointer is NULL");
    return 0;
  }
  for (int j = 0; j < nfield; j++) {
    // MMG5_Scalar / MMG5_Vector / MMG5_Tensor are the only solution types at vertices
    if (!fields || !fields[j] || !(field_size[j] == 1 || field_size[j] == 3 || field_size[j] == 6)) {
      set_err(c, "set_solutions: field %d has size %d (expected 1, 3 or 6)", j, field_size ? field_size[j] : -1);
      return 0;
    }
    if (where == PMMG_HIP_DEVICE && field_size[j] == 6 && ((uintptr_t)fields[j] & 15)) {
      set_err(c, "set_solutions: device tensor field %d must be 16-byte aligned", j);
      return 0;
    }
  }
  if (where == PMMG_HIP_DEVICE && met_size == 6 && ((uintptr_t)met & 15)) {
    set_err(c, "set_solutions: a device tensor metric must be 16-byte aligned");
    return 0;
  }
  size_t np = (size_t)c->bg.np;
  if (np == 0) {
    set_err(c, "set_solutions: call pmmg_hip_set_background first");
    return 0;
  }
  c->met_size = met_size;
  c->nfield = nfield;
  c->fsize.assign(field_size, field_size + nfield);
  c->fin.resize(nfield);
  c->rec = nullptr;
  c->rstride = 0;
  if (where == PMMG_HIP_DEVICE) {
    if (c->carry_slot >= 0) {
      set_err(c, "set_solutions: a carry-over is armed; it takes host-mode (PMMG_HIP_HOST) calls");
      carry_disarm(c);
      return 0;
    }
    c->met = met;
    for (int j = 0; j < nfield; j++) c->fin[j] = fields[j];
    return 1;
  }
  if (c->carry_slot >= 0) return carry_solutions(c, met_size, met, nfield, field_size, fields);
  // host mode: through the copy stream (beside a deferred snapshot)
  if (met_size) {
    if (!copy_stream(c) || !upload(c, c->o_met, met, sizeof(double) * met_size * np, c->cstream)) return 0;
    c->met = (const double *)c->o_met.p;
  }
  c->o_f.resize(nfield);
  for (int j = 0; j < nfield; j++) {
    if (!copy_stream(c) || !upload(c, c->o_f[j], fields[j], sizeof(double) * field_size[j] * np, c->cstream))
      return 0;
    c->fin[j] = (const double *)c->o_f[j].p;
  }
  HIPCK(c, hipStreamSynchronize(c->cstream));
  return 1;
}

int pmmg_hip_set_solutions_packed(pmmg_hip_ctx *c, int met_size, int nfield, const int *field_size,
                                  const double *rec, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if ((met_size != 0 && met_size != 1 && met_size != 6) || nfield < 0 || nfield + (met_size ? 1 : 0) > kMaxSlot ||
      (nfield > 0 && !field_size) || !rec) {
    set_err(c, "set_solutions_packed: invalid arguments (met_size=%d nfield=%d)", met_size, nfield);
    return 0;
  }
  int K = met_size;
  for (int j = 0; j < nfield; j++) {
    if (!(field_size[j] == 1 || field_size[j] == 3 || field_size[j] == 6)) {
      set_err(c, "set_solutions_packed: field %d has size %d (expected 1, 3 or 6)", j, field_size[j]);
      return 0;
    }
    K += field_size[j];
  }
  if (K == 0 || !packed_supported(met_size, nfield, field_size)) {
    set_err(c, "set_solutions_packed: slot layout not supported by the packed records (at most 16 doubles, a "
               "compiled layout); use pmmg_hip_set_solutions");
    return 0;
  }
  if (where == PMMG_HIP_DEVICE && ((uintptr_t)rec & 15)) {
    set_err(c, "set_solutions_packed: device records must be 16-byte aligned");
    return 0;
  }
  const size_t np = (size_t)c->bg.np;
  if (np == 0) {
    set_err(c, "set_solutions_packed: call pmmg_hip_set_background first");
    return 0;
  }
  if (c->carry_slot >= 0) {
    set_err(c, "set_solutions_packed: a carry-over is armed; it takes pmmg_hip_set_solutions (the kept rows are "
               "per-solution arrays)");
    carry_disarm(c);
    return 0;
  }
  c->met_size = met_size;
  c->nfield = nfield;
  c->fsize.assign(field_size, field_size + nfield);
  c->fin.assign(nfield, nullptr);
  c->met = nullptr;
  c->rstride = (K + 1) & ~1;
  if (where == PMMG_HIP_DEVICE) {
    c->rec = rec;
    return 1;
  }
  if (!copy_stream(c) || !upload(c, c->o_rec, rec, sizeof(double) * c->rstride * np, c->cstream)) return 0;
  c->rec = (const double *)c->o_rec.p;
  HIPCK(c, hipStreamSynchronize(c->cstream));
  return 1;
}

// groups with fewer new points take the input order without the coherence
// test: their background stays in the caches, and the binning costs more
// than a numbering's locality (r04g, shuffled numberings: cfg2's 205k points
// 0.19 ms per call in input order, 0.31 Morton-binned; cfg3's 4.1M points
// 2.74 vs 1.89 ms)
constexpr int kSmallGroup = 1 << 20;

static int grid_dim(long long n, int per_cell, int gmax) {
  double g = cbrt((double)n / (double)per_cell);
  int gi = (int)g;
  if (gi < 1) gi = 1;
  if (gi > gmax) gi = gmax;
  return gi;
}

static int blocks_for(long long n, int cap) {
  long long b = (n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

// exhaustive fallbacks of the volume queries (main stream, after the exact
// continuation) and of the surface queries (surface stream, after k_bdy): the
// lists and their counts live on the device, every kernel reads its count
static void launch_vol_fallbacks(pmmg_hip_ctx *c, const Slots &S, const double *xyz_new, int *elem_out,
                                 int8_t *hit_out, hipEvent_t stop = nullptr) {
  const Bg &bg = c->bg;
  hipStream_t s = c->stream;
  DevStats *st = (DevStats *)c->stats.p;
  const int *fb = (const int *)c->fb_vol.p;
  // grids sized by the background (a small group's empty fallback launches cost their dispatch: r04l, cfg2,
  // ~4 us each at 1024 blocks)
  const int gv = (int)std::min<long long>(kFbGridVol, std::max<long long>(64, bg.ne / 16384)) & ~7;
  hipLaunchKernelGGL(k_vol_exhaust_accept, dim3(gv), dim3(kBlock), 0, s, bg, xyz_new, fb, st,
                     (int *)c->best.p, (int *)c->nac.p, (const int *)c->fbg_vol_c.p, (const int *)c->fbg_vol_i.p, S,
                     elem_out, hit_out);
  hipExtLaunchKernelGGL(k_vol_exhaust_closest, dim3(gv), dim3(kBlock), 0, s, nullptr, stop, 0, bg, xyz_new, fb, st,
                        (const int *)c->nac.p, (FbPart *)c->fbp_vol.p, (int *)c->cres.p, S, elem_out, hit_out);
}

static void launch_bdy_fallbacks(pmmg_hip_ctx *c, hipStream_t s, const Slots &S, const double *xyz_new,
                                 int *elem_out, int8_t *hit_out, hipEvent_t stop = nullptr) {
  const Bg &bg = c->bg;
  DevStats *st = (DevStats *)c->stats.p;
  const int *fb = (const int *)c->fb_bdy.p;
  const int gb = (int)std::min<long long>(kFbGridBdy, std::max<long long>(32, bg.nt / 4096)) & ~7;
  hipLaunchKernelGGL(k_bdy_exhaust_accept, dim3(gb), dim3(kBlock), 0, s, bg, xyz_new, fb, st,
                     (int *)c->bbest.p, (int *)c->bnac.p, (const int *)c->fbg_bdy_c.p, (const int *)c->fbg_bdy_i.p, S,
                     elem_out, hit_out);
  hipExtLaunchKernelGGL(k_bdy_exhaust_closest, dim3(gb), dim3(kBlock), 0, s, nullptr, stop, 0, bg, xyz_new, fb, st,
                        (const int *)c->bnac.p, (FbPart *)c->fbp_bdy.p, (int *)c->bcres.p, S, elem_out, hit_out);
}

#ifdef PMMG_HIP_MEASURE
// PMMG_HIP_BRICK=b: the background renumbered by bricks of b^3 seed cells
// (measurement only: pmmg_brick.hpp); the results go nowhere
static int brick_renumber(pmmg_hip_ctx *c, hipStream_t s, const Bg &bg, const Slots &S, const Frame *fr, int g) {
  int lb = 0;
  while ((2 << lb) <= c->brick) lb++;
  const size_t nmax = (size_t)(bg.np > bg.ne ? bg.np : bg.ne);
  size_t nsol = 0;
  for (int j = 0; j < S.n; j++) nsol += (size_t)S.s[j].code;
  if (!ensure(c, c->brk_k, 4 * nmax) || !ensure(c, c->brk_k2, 4 * nmax) || !ensure(c, c->brk_v, 4 * nmax) ||
      !ensure(c, c->brk_v2, 4 * nmax) || !ensure(c, c->brk_vinv, 4 * (size_t)bg.np) ||
      !ensure(c, c->brk_tinv, 4 * (size_t)bg.ne) || !ensure(c, c->brk_xq, 4 * kXqStride * (size_t)bg.np) ||
      !ensure(c, c->brk_xyz, 24 * (size_t)bg.np) || !ensure(c, c->brk_sol, 8 * nsol * (size_t)bg.np + 8) ||
      !ensure(c, c->brk_rec, 32 * (size_t)bg.ne))
    return 0;
  unsigned *k1 = (unsigned *)c->brk_k.p, *k2 = (unsigned *)c->brk_k2.p;
  int *v1 = (int *)c->brk_v.p, *v2 = (int *)c->brk_v2.p;
  int *vinv = (int *)c->brk_vinv.p, *tinv = (int *)c->brk_tinv.p;
  const int kbits = 3 * (10 - lb);
  size_t tmp = 0;
  HIPCK(c, rocprim::radix_sort_pairs(nullptr, tmp, (const unsigned *)k1, k2, (const int *)v1, v2, nmax, 0, kbits, s));
  if (!ensure(c, c->brk_tmp, tmp)) return 0;
  // vertices: keys, sort, inverse, rows
  hipLaunchKernelGGL(k_brick_vkeys, dim3(blocks_for(bg.np, 4096)), dim3(kBlock), 0, s, bg, fr, g, lb, k1, v1);
  HIPCK(c, rocprim::radix_sort_pairs(c->brk_tmp.p, tmp, (const unsigned *)k1, k2, (const int *)v1, v2, (size_t)bg.np, 0,
                                     kbits, s));
  hipLaunchKernelGGL(k_brick_inv, dim3(blocks_for(bg.np, 4096)), dim3(kBlock), 0, s, (const int *)v2,
                     (long long)bg.np, vinv);
  hipLaunchKernelGGL(k_brick_vrows, dim3(blocks_for(bg.np, 4096)), dim3(kBlock), 0, s, bg, (const int *)v2,
                     (int *)c->brk_xq.p, (double *)c->brk_xyz.p);
  size_t off = 0;
  for (int j = 0; j < S.n; j++) {
    hipLaunchKernelGGL(k_brick_srows, dim3(blocks_for((long long)bg.np * S.s[j].code, 4096)), dim3(kBlock), 0, s,
                       S.s[j].in, S.s[j].istride, S.s[j].code, (const int *)v2, (long long)bg.np,
                       (double *)c->brk_sol.p + off * (size_t)bg.np);
    off += (size_t)S.s[j].code;
  }
  // tetra: keys, sort, inverse, records (vertex ids and adjacencies renumbered)
  hipLaunchKernelGGL(k_brick_tkeys, dim3(blocks_for(bg.ne, 4096)), dim3(kBlock), 0, s, bg, fr, g, lb, k1, v1);
  HIPCK(c, rocprim::radix_sort_pairs(c->brk_tmp.p, tmp, (const unsigned *)k1, k2, (const int *)v1, v2, (size_t)bg.ne, 0,
                                     kbits, s));
  hipLaunchKernelGGL(k_brick_inv, dim3(blocks_for(bg.ne, 4096)), dim3(kBlock), 0, s, (const int *)v2, (long long)bg.ne,
                     tinv);
  hipLaunchKernelGGL(k_brick_trec, dim3(blocks_for(bg.ne, 4096)), dim3(kBlock), 0, s, bg, (const int *)v2,
                     (const int *)vinv, (const int *)tinv, (int4 *)c->brk_rec.p);
  HIPCK(c, hipGetLastError());
  return 1;
}
#endif

// The pipeline of one call on device pointers.  It enqueues its kernels on
// the context's two streams and reads nothing back: in auto order mode both
// the Morton binning and the input-order compaction are enqueued, each gated
// on the coherence test's flag on the device (r04), and every fallback kernel
// reads its list's count on the device.
static int run_device(pmmg_hip_ctx *c, int np_new, const double *xyz_new, const uint8_t *pclass, double *met_out,
                      double *const *fields_out, int *elem_out, int8_t *hit_out, double *rec_out = nullptr) {
  Bg bg = c->bg;
  hipStream_t s = c->stream, sb = c->stream2;
  // Measurement build (PMMG_HIP_SRFPRIO=1): a large call runs its second
  // stream (query order, then the surface branch) at the highest priority, so
  // k_bdy's blocks are dispatched ahead of the volume kernel's instead of
  // trailing it (r04o trace: the surface branch ended 0.17 ms after the
  // volume kernel; cfg4 -0.06 ms, r04zh).  Not in the product: once a
  // high-priority stream has existed in the process — even destroyed — the
  // groups call's lanes run at 0.22-0.33 instead of 0.095 ms per cfg2-size
  // group (r04x, r04zg).  The second stream always waits for the main
  // stream's first event, so a call may use either.
  if (c->srf_prio && np_new >= kSmallGroup) {
    if (!c->stream2_hi) {
      int prio_lo = 0, prio_hi = 0;
      (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
      if (hipStreamCreateWithPriority(&c->stream2_hi, hipStreamNonBlocking, prio_hi) != hipSuccess)
        c->stream2_hi = nullptr;
    }
    if (c->stream2_hi) sb = c->stream2_hi;
  }
  Slots S{};
  S.n = 0;
  S.has_met = c->met_size ? 1 : 0;
  if (rec_out && !c->rec) {
    set_err(c, "locate_interp_rec: output records need packed input records (pmmg_hip_set_solutions_packed)");
    return 0;
  }
  if (c->met_size) {
    if (!met_out && !rec_out) {
      set_err(c, "locate_interp: met_out is NULL");
      return 0;
    }
    S.s[S.n++] = Slot{c->met, met_out, c->met_size, c->met_size, c->met_size};
  }
  for (int j = 0; j < c->nfield; j++) {
    if (!rec_out && (!fields_out || !fields_out[j])) {
      set_err(c, "locate_interp: fields_out[%d] is NULL", j);
      return 0;
    }
    S.s[S.n++] = Slot{c->fin[j], rec_out ? nullptr : fields_out[j], c->fsize[j], c->fsize[j], c->fsize[j]};
  }
  if (c->rec) { // packed records: every slot reads its columns of the record
    S.rec = c->rec;
    int off = 0;
    for (int j = 0; j < S.n; j++) {
      S.s[j].in = c->rec + off;
      S.s[j].istride = c->rstride;
      if (rec_out) { // and writes its columns of the new point's output record
        S.s[j].out = rec_out + off;
        S.s[j].ostride = c->rstride;
      }
      off += S.s[j].code;
    }
    S.rec_out = rec_out;
  }
  const VolPick vpick = pick_layout(S, c->pack_passes);
  if (!vpick.fn) {
    set_err(c, "locate_interp: no packed-record kernel for this slot layout");
    return 0;
  }
  const bool vsplit = S.n > 0 && vpick.ifn && (c->vol_split < 0 ? np_new >= kSmallGroup : c->vol_split == 1);
  LocBuf lb{nullptr, nullptr, nullptr};
  if (vsplit) {
    if (!ensure(c, c->locv, 16 * (size_t)np_new) || !ensure(c, c->locp, 32 * (size_t)np_new)) return 0;
    lb = LocBuf{(nti4 *)c->locv.p, (ntd2 *)c->locp.p, (ntd2 *)c->locp.p + np_new};
    if (!c->stream_i) HIPCK(c, hipStreamCreateWithFlags(&c->stream_i, hipStreamNonBlocking));
    for (auto &row : c->ev_chunk)
      for (hipEvent_t &e : row)
        if (!e) HIPCK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!c->ev_interp) HIPCK(c, hipEventCreateWithFlags(&c->ev_interp, hipEventDisableTiming));
  }
  const VolFn vol_fn = vsplit ? kVolWalk : vpick.fn;
  const int g = grid_dim(bg.ne, c->tpc, 1024);
  const int gs = bg.nt <= 0 ? 1 : (c->srf_g > 0 ? c->srf_g : grid_dim((long long)bg.nt * c->srf_mult, 2, 1024));
  const int gb = 1 << kBinBitsAxis;
  const size_t nq = (size_t)np_new;
  const long long ng = (long long)g * g * g, nsg = bg.nt > 0 ? (long long)gs * gs * gs : 0;
  const long long ncls = (long long)(nq / kScanChunk + 1);
  if (!ensure(c, c->frame, sizeof(Frame)) || !ensure(c, c->stats, sizeof(DevStats) + kStatParts * sizeof(StatPart)) ||
      !ensure(c, c->grid, 8 * (size_t)ng) || !ensure(c, c->sgrid, 8 * (size_t)nsg) || !ensure(c, c->order_v, 4 * nq) ||
      !ensure(c, c->order_b, 4 * nq) || !ensure(c, c->cont, sizeof(ContEntry) * nq) ||
      !ensure(c, c->bkeys, 4 * nq) || !ensure(c, c->bkeys2, 4 * nq) || !ensure(c, c->bvals, 4 * nq) ||
      !ensure(c, c->qs, 24 * nq) || !ensure(c, c->cls_cnt, 4 * (size_t)ncls) || 
      !ensure(c, c->fb_vol, 4 * nq) || !ensure(c, c->fb_bdy, 4 * nq) || !ensure(c, c->best, 4 * nq) ||
      !ensure(c, c->nac, 4 * nq) || !ensure(c, c->cres, 4 * nq) || !ensure(c, c->bbest, 4 * nq) ||
      !ensure(c, c->bnac, 4 * nq) || !ensure(c, c->bcres, 4 * nq) ||
      !ensure(c, c->fbp_vol, sizeof(FbPart) * (size_t)kFbPartCap) ||
      !ensure(c, c->fbp_bdy, sizeof(FbPart) * 256 * (size_t)kFbGridBdy) ||
      !ensure(c, c->fbg_vol_c, 4 * (size_t)(kFbCells + 1)) || !ensure(c, c->fbg_vol_u, 4 * (size_t)kFbCells) ||
      !ensure(c, c->fbg_vol_i, 4 * nq) || !ensure(c, c->fbg_bdy_c, 4 * (size_t)(kFbCells + 1)) ||
      !ensure(c, c->fbg_bdy_u, 4 * (size_t)kFbCells) || !ensure(c, c->fbg_bdy_i, 4 * nq))
    return 0;
  if (!ensure(c, c->xq, sizeof(int) * kXqStride * (size_t)bg.np) || !ensure(c, c->oflag, 2 * sizeof(int)) ||
      !ensure(c, c->cohd, sizeof(double) * kCohSamples) ||
      !ensure(c, c->axh, sizeof(int) * 3 * kMapBins * (size_t)kHistBlocks))
    return 0;
  bg.xq = (const int *)c->xq.p;
  Frame *fr = (Frame *)c->frame.p;
  DevStats *st = (DevStats *)c->stats.p;
  unsigned long long *grid = (unsigned long long *)c->grid.p;
  unsigned long long *sgrid = (unsigned long long *)c->sgrid.p;
  int *order_v = (int *)c->order_v.p, *order_b = (int *)c->order_b.p;
  int force = (c->options & PMMG_HIP_OPT_SORT) ? 1 : (c->options & PMMG_HIP_OPT_NOSORT) ? 0 : -1;
  if (force < 0 && np_new < kSmallGroup) force = 0;
  // r06: a large auto-order call reads the decision back once k_bbox is done (the host waits while the device
  // runs the fixed-point copy and the seed grid, ~0.4 ms at cfg4) and enqueues only the chosen order's
  // kernels.  With both orders enqueued and gated on the device, the input order's volume kernel waited for
  // the ~19 gated binning launches (each dispatched only when the preparation kernels left a slot free: they
  // ended 20-55 us after the seed grid, profiles/r06i, r06k), or, below 2^23 queries, the other order's
  // volume launch returned at once in 40-64k one-wave blocks (~35-55 us of dispatch on the main stream).
  const bool host_order = force < 0 && c->host_order;
  if (host_order && !c->flag_host) {
    void *p = nullptr;
    HIPCK(c, hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
    c->flag_host = (int *)p;
    void *d = nullptr;
    HIPCK(c, hipHostGetDevicePointer(&d, p, 0));
    c->flag_host_dev = (int *)d;
  }
  if (host_order) c->flag_host[0] = -1;

  // ---- frame (main stream).  The call's events ride on its kernels' dispatches where a kernel is at hand
  // (hipExtLaunchKernelGGL start / stop events): a separate marker between two kernels of a stream cost the
  // device ~4 us, an event on the dispatch ~1.7 (tools/calib/ext_event.hip, profiles/r06zj)
  // seed grids: cleared here unless the previous call left them clean (a
  // large grid is refilled at the end of the call that used it, beside the
  // other stream's tail: r05, cfg4 k_reset 32 us -> the stats only)
  const long long ng_clr = (c->grid.p == c->grid_clean_p && ng <= c->grid_clean_n) ? 0 : ng;
  const long long nsg_clr = (c->sgrid.p == c->sgrid_clean_p && nsg <= c->sgrid_clean_n) ? 0 : nsg;
  c->grid_clean_n = c->sgrid_clean_n = 0; // dirty until this call's refill is enqueued
  // the input order's surface list needs only the zeroed counters (and the coherence flag), not the frame
  // (r06: EV_RESET is waited for only in a forced order, EV_VOL0 / EV_VOL only when a kernel separates them
  // from EV_PREP / EV_WALK)
  hipExtLaunchKernelGGL(k_reset, dim3(blocks_for(ng_clr > nsg_clr ? ng_clr : nsg_clr, 2048)), dim3(kBlock), 0, s,
                        c->ev[EV_START], force >= 0 ? c->ev[EV_RESET] : nullptr, 0, fr, st, grid, ng_clr, sgrid,
                        nsg_clr, (int *)c->oflag.p, force, c->bin_bits);
  // bbox (its last block finalises the frame), the seed grid's axis maps
  // (auto order: the queries' coherence test rides along, its flag read by the order and volume kernels)
  // the second stream needs the frame only (lo, inv_bin, inv_srf), not the
  // axis maps (r04: EV_FRAME moved here from after k_axis_map)
  hipExtLaunchKernelGGL(k_bbox, dim3(std::max(force < 0 ? kCohBlocks : 1, blocks_for(bg.np / c->bbox_stride + 1, 256))),
                        dim3(kBlock), 0, s, nullptr, c->ev[EV_FRAME], 0, (const double *)bg.xyz, bg.np, fr,
                        c->bbox_stride, g, gs, gb, xyz_new, np_new, force < 0 ? (int *)c->oflag.p : nullptr,
                        (double *)c->cohd.p, host_order ? c->flag_host_dev : nullptr);
  // fixed-point vertex copy + the axis histograms (first kHistBlocks blocks), then the axis maps.
  // quant_side (r06, large calls): the histograms alone on the main stream, the copy on a stream of its own
  // beside the seed grid, which then takes its centroids from the fp64 rows; the volume kernel waits for both
  const bool quant_side = c->quant_side && np_new >= kSmallGroup;
  if (quant_side) {
    if (!c->stream_f) HIPCK(c, hipStreamCreateWithFlags(&c->stream_f, hipStreamNonBlocking));
    HIPCK(c, hipStreamWaitEvent(c->stream_f, c->ev[EV_FRAME], 0));
    hipLaunchKernelGGL(k_quantize, dim3(blocks_for(3LL * bg.np, 8192)), dim3(kBlock), 0, c->stream_f, bg.xyz,
                       (long long)bg.np, (const Frame *)fr, (int *)c->xq.p, c->hist_stride, (int *)nullptr);
    HIPCK(c, hipEventRecord(c->ev[EV_QUANT], c->stream_f));
    hipLaunchKernelGGL(k_axis_hist, dim3(kHistBlocks), dim3(kBlock), 0, s, bg.xyz, (long long)bg.np,
                       (const Frame *)fr, c->hist_stride, (int *)c->axh.p);
  } else {
    hipLaunchKernelGGL(k_quantize, dim3(std::max(kHistBlocks, blocks_for(3LL * bg.np, 8192))), dim3(kBlock), 0, s,
                       bg.xyz, (long long)bg.np, (const Frame *)fr, (int *)c->xq.p, c->hist_stride, (int *)c->axh.p);
  }
  hipLaunchKernelGGL(k_axis_map, dim3(3), dim3(kBlock), 0, s, (const int *)c->axh.p, fr, g);
  HIPCK(c, hipGetLastError());

  // ---- query order (second stream, concurrent with the seed grid), after
  // the frame.  (r04: the axis maps moved here beside the fixed-point copy
  // cost 10 groups 0.11 -> 0.25 ms per group and the 8-way rank +0.02 ms for
  // -0.0 at cfg4, `profiles/r04s`: not kept)
  HIPCK(c, hipStreamWaitEvent(sb, c->ev[force < 0 ? EV_FRAME : EV_RESET], 0)); // (the order flag)
  // (EV_SB0: the start of the surface list's first kernel when there is one, launch_cls)
  if (force == 1 || bg.nt <= 0) HIPCK(c, hipEventRecord(c->ev[EV_SB0], sb));
  // the Morton binning on a third stream (r05, `profiles/r05m`: on the second stream its ~19 launches, each
  // returning at once when the coherence test picks input order, held the 8-way rank's volume kernel 86 us
  // behind the seed grid)
  hipStream_t sc = sb;
  if (force != 0) {
    if (c->stream3_mode == 1 && !c->stream3 &&
        hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking) != hipSuccess)
      c->stream3 = nullptr;
    if (c->stream3) sc = c->stream3;
    HIPCK(c, hipStreamWaitEvent(sc, c->ev[EV_FRAME], 0)); // (the frame and the order flag)
  }
  // auto mode with the binning on its own stream (split): the input order's lists (EV_ORDER, second stream)
  // and the Morton order's (EV_ORDER2, third stream) are waited for separately, each by the launch of the
  // volume / surface kernel for its order (the other launch returns at once): a call in input order no longer
  // waits for the ~19 binning launches, which return at once but take ~130 us in a row (r05n, 8-way rank).
  // Below 2^23 queries: a larger call's seed grid outlasts the binning chain anyway (cfg4's preparation
  // 0.41 ms) and keeps one volume launch per call.
  bool split = force < 0 && sc != sb && np_new < (1 << 23);
  HIPCK(c, hipGetLastError());

  // ---- seed grid (main stream): volume seeds
  {
    const long long nsamp = ng < bg.ne ? ng : bg.ne;
    // kSeedBatch samples per thread in flight together (r05m: one per thread, the 8-way rank's 1.65M samples
    // took 107 us — the grid's latency in rounds of waves — where cfg4's 12.6M take 262 us)
    hipExtLaunchKernelGGL(k_seed_vol, dim3((blocks_for((nsamp + kSeedBatch - 1) / kSeedBatch, 8192) + 7) & ~7),
                          dim3(kBlock), 0, s, nullptr, quant_side ? nullptr : c->ev[EV_PREP], 0, bg, fr, grid, g,
                          nsamp, c->seed_lanes, c->seed_v0, quant_side ? bg.xyz : (const double *)nullptr);
    if (quant_side) { // (the walk reads the fixed-point copy)
      HIPCK(c, hipStreamWaitEvent(s, c->ev[EV_QUANT], 0));
      HIPCK(c, hipEventRecord(c->ev[EV_PREP], s));
    }
  }
  HIPCK(c, hipGetLastError());

  // ---- query order (second stream, after the frame): the kernels of both
  // orders, each gated on the coherence test's flag (k_bbox's extra block) on the device — no host read.
  // Forced orders enqueue only theirs; a small group (below kSmallGroup
  // queries: its background and solutions stay in the Infinity Cache, where
  // a numbering's locality matters little) takes the input order untested.
  const int *flag = (const int *)c->oflag.p;
#ifdef PMMG_HIP_MEASURE
  if (c->set_order) hipLaunchKernelGGL(k_set_order, dim3(1), dim3(1), 0, s, st, force > 0 ? 1 : 0, c->bin_bits);
#endif
  // input order: the surface points in input order (stable compaction:
  // per-block counts, their scan, the scatter; rocPRIM's select took 0.2 ms
  // longer here, r03o)
  // (EV_SB0 on its first kernel; EV_ORDER on its last with order_end; returns whether EV_ORDER was recorded)
  auto launch_cls = [&](bool order_end) -> bool {
    if (force == 1 || bg.nt <= 0) return false;
    int *bc = (int *)c->cls_cnt.p;
    hipExtLaunchKernelGGL(k_cls_count, dim3((unsigned)ncls), dim3(kBlock), 0, sb, c->ev[EV_SB0], nullptr, 0,
                          pclass, (long long)np_new, (int)PMMG_PT_BDY, bc, flag, 0);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, sb, bc, (int)ncls, &st->nbdy, flag, 0);
    hipExtLaunchKernelGGL(k_cls_scatter, dim3((unsigned)ncls), dim3(kBlock), 0, sb, nullptr,
                          order_end ? c->ev[EV_ORDER] : nullptr, 0, pclass, (long long)np_new, (int)PMMG_PT_BDY,
                          (const int *)bc, order_b, flag, 0);
    return order_end;
  };
  // Morton order: stable LSD radix sort of the keys (<= 3 * 7 + 2 bits) in 3 passes of 8 bits
  // (pmmg_sort.hpp); the key kernel writes the first pass's digit table
  auto launch_morton = [&]() -> int {
    if (force == 0 || np_new <= 0) return 1;
    const int ntile = (int)((np_new + kRsTile - 1) / kRsTile);
    const long long nh = 256LL * ntile;
    const int nch = (int)((nh + kScanChunk - 1) / kScanChunk);
    if (!ensure(c, c->bvals2, 4 * nq) || !ensure(c, c->rs_hist, 4 * (size_t)nh) || !ensure(c, c->rs_csum, 4 * (size_t)nch))
      return 0;
    unsigned *k0 = (unsigned *)c->bkeys.p, *k1 = (unsigned *)c->bkeys2.p;
    int *v0 = (int *)c->bvals.p, *v1 = (int *)c->bvals2.p, *hist = (int *)c->rs_hist.p, *csum = (int *)c->rs_csum.p;
    const int tgrid = std::min(ntile, kRsGrid);
    hipLaunchKernelGGL(k_bin_keys, dim3(tgrid), dim3(kBlock), 0, sc, xyz_new, pclass, np_new, (const Frame *)fr, flag,
                       k0, v0, st, kRsTile, ntile, hist);
    for (int pass = 0; pass < 3; pass++) {
      const unsigned *kin = pass == 1 ? k1 : k0;
      const int *vin = pass == 1 ? v1 : v0;
      unsigned *kout = pass == 1 ? k0 : k1;
      int *vout = pass == 1 ? v0 : (pass == 0 ? v1 : order_v);
      if (pass > 0)
        hipLaunchKernelGGL(k_rs_hist, dim3(tgrid), dim3(kBlock), 0, sc, kin, np_new, 8 * pass, ntile, hist, flag, 1);
      hipLaunchKernelGGL(k_rs_scan_local, dim3(nch), dim3(kBlock), 0, sc, hist, (int)nh, csum, flag, 1);
      hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, sc, csum, nch, (int *)nullptr, flag, 1);
      hipLaunchKernelGGL(k_rs_scan_add, dim3(nch), dim3(kBlock), 0, sc, hist, (int)nh, (const int *)csum, flag, 1);
      hipLaunchKernelGGL(k_rs_scatter, dim3(tgrid), dim3(kBlock), 0, sc, kin, vin, np_new, 8 * pass, ntile,
                         (const int *)hist, kout, vout, flag, 1);
    }
    hipLaunchKernelGGL(k_bin_split, dim3(blocks_for(np_new, 4096)), dim3(kBlock), 0, sc, (const int *)order_v, xyz_new,
                       np_new, order_b, c->bin_qs ? (double *)c->qs.p : nullptr, (const DevStats *)st, flag);
    return 1;
  };
  // one round of the grid for up to 1M surface points (static split: a
  // second, nearly empty round doubled the surface branch alone)
  unsigned long long *wt = nullptr;
#ifdef PMMG_HIP_MEASURE
  if (c->wave_time) {
    const size_t nw = (size_t)8 * blocks_for((np_new + 7) / 8, c->bdy_bpx) * (kBlock / 64);
    if (!ensure(c, c->wt, 32 * nw)) return 0;
    HIPCK(c, hipMemsetAsync(c->wt.p, 0, 32 * nw, sb));
    wt = (unsigned long long *)c->wt.p;
    c->wt_n = nw;
  }
#endif
  // k_bdy's blocks: kBlock threads, or one wave each (bdy_wave), so that they fit into the single-wave
  // slots the volume kernel's one-wave blocks leave while it runs beside them
  const int bdy_tpb = c->bdy_wave ? 64 : kBlock;
  auto bdy = [&](int want) {
    hipLaunchKernelGGL(k_bdy, dim3(8 * blocks_for((np_new + 7) / 8, c->bdy_bpx) * (kBlock / bdy_tpb)), dim3(bdy_tpb),
                       0, sb, bg,
                       (const Frame *)fr, (const unsigned long long *)sgrid, gs, xyz_new, (const int *)order_b, S, elem_out,
                       hit_out, (int *)c->fb_bdy.p, st, c->maxstep, c->bdy_dyn, FbInit{(int *)c->bbest.p},
                       FbGridBufs{(int *)c->fbg_bdy_c.p, (int *)c->fbg_bdy_u.p, (int *)c->fbg_bdy_i.p}, flag, want, wt);
  };
  // ---- surface branch (second stream, after the order): seeds, k_bdy
  // (r05ae: the surface seeds moved before the wait for the volume seed grid, beside it: preparation
  // +0.03 ms at cfg4, +0.17 for the Mmg-like numbering, the 8-way rank +0.04 — not kept)
  auto srf_head = [&]() {
    if (c->srf_solo > 0 || (c->srf_solo < 0 && np_new >= kSmallGroup))
      HIPCK(c, hipStreamWaitEvent(sb, c->ev[EV_PREP], 0));
    if (bg.nt <= 0) HIPCK(c, hipEventRecord(c->ev[EV_BDY0], sb)); // (else the start of the surface seeds)
    if (bg.nt > 0) {
      if (force == 0) HIPCK(c, hipStreamWaitEvent(sb, c->ev[EV_FRAME], 0)); // (the surface seeds need the frame)
      hipExtLaunchKernelGGL(k_seed_srf, dim3(blocks_for(bg.nt, 4096) * (kBlock / bdy_tpb)), dim3(bdy_tpb), 0, sb,
                            c->ev[EV_BDY0], nullptr, 0, bg, (const Frame *)fr, sgrid, gs);
      if (c->vol_wait_seed) HIPCK(c, hipEventRecord(c->ev[EV_SRFSEED], sb));
    }
    return 1;
  };
  auto srf_tail = [&]() {
    bool rec = false; // EV_BDY1 recorded by the branch's last launch
    const bool fill = nsg >= kRefillCells;
    if (bg.nt > 0) {
      if (!c->no_fb) {
        hipLaunchKernelGGL(k_fb_grid, dim3(1), dim3(bdy_tpb), 0, sb, xyz_new, (const int *)c->fb_bdy.p, st, 1,
                           FbGridBufs{(int *)c->fbg_bdy_c.p, (int *)c->fbg_bdy_u.p, (int *)c->fbg_bdy_i.p});
        // one-wave surface branch: its exhaustive kernels (blocks of kBlock threads, which a running volume
        // kernel's one-wave blocks would keep waiting for four free slots) run on the main stream after the
        // volume ones
        if (c->bdy_wave) HIPCK(c, hipEventRecord(c->ev[EV_BDYFB], sb));
        else launch_bdy_fallbacks(c, sb, S, xyz_new, elem_out, hit_out, fill ? nullptr : c->ev[EV_BDY1]);
        rec = !c->bdy_wave && !fill;
      }
      HIPCK(c, hipGetLastError());
      if (fill) { // the surface grid refilled for the next call (see k_reset above)
        hipExtLaunchKernelGGL(k_fill64, dim3(blocks_for((nsg + 1) / 2, 2048) * (kBlock / bdy_tpb)), dim3(bdy_tpb), 0,
                              sb, nullptr, c->ev[EV_BDY1], 0, sgrid, nsg, ~0ULL);
        rec = true;
        c->sgrid_clean_p = c->sgrid.p;
        c->sgrid_clean_n = nsg;
      }
    }
    if (!rec) HIPCK(c, hipEventRecord(c->ev[EV_BDY1], sb));
    return 1;
  };
  // ---- volume (main stream): walk + exact test + interpolation in one
  // kernel, then the exact continuation of the few queries it did not settle
  const bool fuse_cont = c->fuse_cont && !vsplit;
  const ContArgs ca{(int *)c->fb_vol.p, FbInit{(int *)c->best.p}, c->maxstep, fuse_cont ? 1 : 0};
  // (stop: an event the launch records, EV_WALK when it is the call's only volume launch)
  auto vol = [&](int want, hipEvent_t stop) {
    // (measurement build; a plain call: HIPCK's `return 0` would give this void lambda a return type)
    if (c->vol_wait_seed && bg.nt > 0 && want <= 0) (void)hipStreamWaitEvent(s, c->ev[EV_SRFSEED], 0);
    const int nb = (np_new + 63) / 64;
    if (!vsplit) {
      hipExtLaunchKernelGGL(vol_fn, dim3(nb), dim3(64), 0, s, nullptr, stop, 0, bg, (const Frame *)fr,
                            (const unsigned long long *)grid, g, xyz_new, pclass, (const int *)order_v,
                            c->bin_qs ? (const double *)c->qs.p : nullptr, np_new, (ContEntry *)c->cont.p, st, S,
                            elem_out, hit_out, c->filter_steps, flag, c->xcd_run, c->pad, want, lb, 0, ca);
      return;
    }
    // split stage: walk chunk j (main stream), then its interpolation on stream_i, beside walk chunk j + 1
    // (chunks of whole XCD runs)
    const int run = 8 * std::max(1, c->xcd_run);
    const int per = std::max(run, (nb + c->vol_chunks - 1) / c->vol_chunks / run * run);
    const int ixr = c->ixcd_run >= 0 ? c->ixcd_run : c->xcd_run;
    const int w = want > 0 ? 1 : 0;
    for (int j = 0, b0 = 0; b0 < nb; j++, b0 += per) {
      const int nbj = std::min(per, nb - b0);
      hipLaunchKernelGGL(vol_fn, dim3(nbj), dim3(64), 0, s, bg, (const Frame *)fr, (const unsigned long long *)grid,
                         g, xyz_new, pclass, (const int *)order_v, c->bin_qs ? (const double *)c->qs.p : nullptr,
                         np_new, (ContEntry *)c->cont.p, st, S, elem_out, hit_out, c->filter_steps, flag,
                         c->xcd_run, c->pad, want, lb, b0, ca);
      hipEvent_t ej = c->ev_chunk[w][std::min(j, (int)pmmg_hip_ctx::kMaxVolChunks - 1)];
      (void)hipEventRecord(ej, s);
      (void)hipStreamWaitEvent(c->stream_i, ej, 0);
      hipLaunchKernelGGL(vpick.ifn, dim3(nbj), dim3(64), 0, c->stream_i, lb, (const int *)order_v,
                         (const DevStats *)st, np_new, S, flag, ixr, want, b0);
    }
  };
  // host_order: the launches that do not depend on the order (the input order's surface list, gated on the
  // device flag; the surface seeds) go out before the host waits for the decision, so that after it only the
  // chosen order's kernels are enqueued, the volume kernel first (r06ze: the device idled ~20 us between the
  // seed grid and the volume kernel of an 8-way rank while the host enqueued ~10 launches ahead of it)
  const bool pre = host_order;
  if (pre) {
    if (!launch_cls(true)) HIPCK(c, hipEventRecord(c->ev[EV_ORDER], sb));
    if (!srf_head()) return 0;
    HIPCK(c, hipGetLastError());
    // the decision, written by k_bbox's last block (coherence_final); from here on a forced order
    HIPCK(c, hipEventSynchronize(c->ev[EV_FRAME]));
    const int f = __atomic_load_n(&c->flag_host[0], __ATOMIC_ACQUIRE);
    if (f != 0 && f != 1) {
      set_err(c, "locate_interp: the query order decision did not arrive (%d)", f);
      return 0;
    }
    force = f;
    split = false; // (the order is known: only its kernels are enqueued, no gated launches of the other)
  }
  if (split) {
    // Host enqueue order (r05q trace): the input order's kernels first — the surface list, the surface
    // seeds and walk, the volume kernel — then the ~19 binning launches and the Morton order's launches.
    // Enqueued after the binning chain, the input order's volume kernel started ~200 us after the seed grid
    // had finished: the host was still enqueueing (~8 us per launch), the device idle.
    if (!launch_cls(true)) HIPCK(c, hipEventRecord(c->ev[EV_ORDER], sb));
    if (!srf_head()) return 0;
    if (bg.nt > 0) bdy(0);
    c->ev_vol0 = EV_VOL0;
    HIPCK(c, hipEventRecord(c->ev[EV_VOL0], s));
    vol(0, nullptr);
    if (!launch_morton()) return 0;
    HIPCK(c, hipGetLastError());
    HIPCK(c, hipEventRecord(c->ev[EV_ORDER2], sc));
    if (bg.nt > 0) {
      HIPCK(c, hipStreamWaitEvent(sb, c->ev[EV_ORDER2], 0));
      bdy(1);
    }
    if (!srf_tail()) return 0;
    HIPCK(c, hipStreamWaitEvent(s, c->ev[EV_ORDER2], 0));
    vol(1, nullptr);
  } else {
    // (EV_ORDER on the surface list's last kernel unless the Morton lists may follow on the same stream;
    // EV_ORDER2 is waited for only when the order is Morton)
    const bool ord = !pre && launch_cls(force == 0);
    if (!launch_morton()) return 0;
    HIPCK(c, hipGetLastError());
    if (!pre && !ord) HIPCK(c, hipEventRecord(c->ev[EV_ORDER], sb));
    if (force != 0) HIPCK(c, hipEventRecord(c->ev[EV_ORDER2], sc)); // (sc == sb: the same point)
    // the volume kernel reads the order branch's lists only in Morton order (or when it may be chosen); in
    // forced input order its queries are the input's volume points and the wait is dropped (r05: the
    // cross-stream wait was ~20 us of a small group's main chain)
    bool vol_first = pre && !c->bdy_first;
#ifdef PMMG_HIP_MEASURE
    vol_first = vol_first && c->brick <= 0;
#endif
    // the volume kernel right after the seed grid (input order, nothing to wait for, nothing launched on the
    // main stream in between): the stage opens at EV_PREP
    bool vol_direct = force == 0 && !c->bdy_first;
#ifdef PMMG_HIP_MEASURE
    vol_direct = vol_direct && c->brick <= 0 && !c->set_order && !c->quant_side;
#endif
    c->ev_vol0 = vol_direct ? EV_PREP : EV_VOL0;
    auto vol_main = [&]() {
      if (force < 0) (void)hipStreamWaitEvent(s, c->ev[EV_ORDER], 0);
      if (force != 0 && sc != sb) (void)hipStreamWaitEvent(s, c->ev[EV_ORDER2], 0);
      if (c->bdy_first) (void)hipStreamWaitEvent(s, c->ev[EV_BDY1], 0);
      if (c->ev_vol0 == EV_VOL0) (void)hipEventRecord(c->ev[EV_VOL0], s);
      vol(-1, vsplit ? nullptr : c->ev[EV_WALK]);
    };
    if (vol_first) vol_main();
    if (sc != sb && force != 0) HIPCK(c, hipStreamWaitEvent(sb, c->ev[EV_ORDER2], 0)); // the Morton surface list
    if (!pre && !srf_head()) return 0;
    if (c->bdy_after && vol_first) HIPCK(c, hipStreamWaitEvent(sb, c->ev[EV_WALK], 0));
    if (bg.nt > 0) bdy(-1);
    if (!srf_tail()) return 0;
#ifdef PMMG_HIP_MEASURE
    if (c->brick > 0 && !brick_renumber(c, s, bg, S, fr, g)) return 0;
#endif
    if (!vol_first) vol_main();
    HIPCK(c, hipGetLastError());
  }
  if (split || vsplit) HIPCK(c, hipEventRecord(c->ev[EV_WALK], s)); // (else recorded by the volume launch)
  // the volume seed grid refilled for the next call as soon as the volume kernel is done with it, on its own
  // stream beside the main stream's tail (the exact continuation, the fallbacks: latency-bound) and the
  // surface stream's; r06: at the end of the main stream it added ~36 us to a cfg4 call (r05ao: on the
  // surface stream right after the volume kernel it ran behind k_bdy's tail instead)
  const bool refill = ng >= kRefillCells;
  if (refill) {
    if (!c->stream_f) HIPCK(c, hipStreamCreateWithFlags(&c->stream_f, hipStreamNonBlocking));
    HIPCK(c, hipStreamWaitEvent(c->stream_f, c->ev[EV_WALK], 0));
    hipExtLaunchKernelGGL(k_fill64, dim3(blocks_for((ng + 1) / 2, 2048)), dim3(kBlock), 0, c->stream_f, nullptr,
                          c->ev[EV_FILL], 0, grid, ng, ~0ULL);
    HIPCK(c, hipGetLastError());
    c->grid_clean_p = c->grid.p;
    c->grid_clean_n = ng;
  }
  // (8 x 64 one-wave blocks for a large call; fewer for a small group, whose continuations are a few hundred)
  const int wx = (int)std::min<long long>(64, std::max<long long>(2, (long long)np_new / 65536));
  if (!fuse_cont) // (continued inside the volume kernel otherwise: ContArgs)
    hipLaunchKernelGGL(k_vol_walk_exact, dim3(8 * wx), dim3(64), 0, s, bg, xyz_new, (int *)c->fb_vol.p,
                       (const ContEntry *)c->cont.p, st, S, elem_out, hit_out, c->maxstep, FbInit{(int *)c->best.p},
                       FbGridBufs{(int *)c->fbg_vol_c.p, (int *)c->fbg_vol_u.p, (int *)c->fbg_vol_i.p});
  HIPCK(c, hipGetLastError());
  if (vsplit) { // the volume stage ends with the interpolation's last chunk
    HIPCK(c, hipEventRecord(c->ev_interp, c->stream_i));
    HIPCK(c, hipStreamWaitEvent(s, c->ev_interp, 0));
  }
  c->ev_vol = (fuse_cont && !vsplit) ? EV_WALK : EV_VOL;
  if (c->ev_vol == EV_VOL) HIPCK(c, hipEventRecord(c->ev[EV_VOL], s));
  // ---- exhaustive fallbacks of the volume queries (lists and counts on the
  // device; the surface ones ran on the surface stream after k_bdy): the
  // list's query grid, then the searches
  const bool bdy_fb_main = !c->no_fb && c->bdy_wave && bg.nt > 0;
  if (!c->no_fb) {
    hipLaunchKernelGGL(k_fb_grid, dim3(1), dim3(kBlock), 0, s, xyz_new, (const int *)c->fb_vol.p, st, 0,
                       FbGridBufs{(int *)c->fbg_vol_c.p, (int *)c->fbg_vol_u.p, (int *)c->fbg_vol_i.p});
    launch_vol_fallbacks(c, S, xyz_new, elem_out, hit_out, bdy_fb_main ? nullptr : c->ev[EV_JOIN]);
  }
  if (bdy_fb_main) {
    HIPCK(c, hipStreamWaitEvent(s, c->ev[EV_BDYFB], 0));
    launch_bdy_fallbacks(c, s, S, xyz_new, elem_out, hit_out);
  }
  HIPCK(c, hipGetLastError());
  if (c->no_fb || bdy_fb_main) HIPCK(c, hipEventRecord(c->ev[EV_JOIN], s)); // (else the last fallback's stop)
  HIPCK(c, hipStreamWaitEvent(s, c->ev[EV_BDY1], 0));
  if (refill) HIPCK(c, hipStreamWaitEvent(s, c->ev[EV_FILL], 0));
  HIPCK(c, hipEventRecord(c->ev[EV_END], s));
  c->pending = true;
  return 1;
}

static int collect_stats(pmmg_hip_ctx *c, pmmg_hip_stats *out) {
#ifdef PMMG_HIP_MEASURE
  if (c->wave_time && c->wt_n) { // k_bdy's per-wave records of the call, appended to PMMG_HIP_WAVETIME_OUT
    std::vector<unsigned long long> w(4 * c->wt_n);
    HIPCK(c, ctx_d2h(c, w.data(), c->wt.p, 8 * w.size()));
    const char *path = getenv("PMMG_HIP_WAVETIME_OUT");
    if (FILE *f = path ? fopen(path, "ab") : nullptr) {
      fwrite(w.data(), 8, w.size(), f);
      fclose(f);
    }
    c->wt_n = 0;
  }
#endif
  DevStats h;
  int order[2] = {0, 0}; // the call's query order, decided on the device
  HIPCK(c, ctx_d2h(c, order, c->oflag.p, sizeof(order)));
  std::vector<StatPart> parts(kStatParts);
  HIPCK(c, ctx_d2h(c, &h, c->stats.p, sizeof(DevStats)));
  HIPCK(c, ctx_d2h(c, parts.data(), (const DevStats *)c->stats.p + 1, kStatParts * sizeof(StatPart)));
  unsigned long long cnt[kNumCnt] = {0}, steps = 0, stepmax = 0;
  for (const StatPart &pt : parts) {
    for (int j = 0; j < kNumCnt; j++) cnt[j] += pt.cnt[j];
    steps += pt.steps;
    if (pt.stepmax > stepmax) stepmax = pt.stepmax;
  }
  memset(out, 0, sizeof(*out));
  out->nvol = order[0] == 1 ? (int64_t)h.nvol : (int64_t)cnt[kCntVolQueries];
  out->nbdy = h.nbdy;
  out->nvol_walk = (int64_t)cnt[PMMG_HIT_VOL_WALK];
  out->nvol_exhaust = (int64_t)cnt[PMMG_HIT_VOL_EXHAUST];
  out->nvol_closest = (int64_t)cnt[PMMG_HIT_VOL_CLOSEST];
  out->nvol_exact = (int64_t)cnt[kCntExact];
  out->nbdy_face = (int64_t)cnt[PMMG_HIT_BDY_FACE];
  out->nbdy_edge = (int64_t)cnt[PMMG_HIT_BDY_EDGE];
  out->nbdy_vertex = (int64_t)cnt[PMMG_HIT_BDY_VERTEX];
  out->nbdy_wedge = (int64_t)cnt[PMMG_HIT_BDY_WEDGE];
  out->nbdy_cone = (int64_t)cnt[PMMG_HIT_BDY_CONE];
  out->nbdy_exhaust = (int64_t)cnt[PMMG_HIT_BDY_EXHAUST];
  out->nbdy_stale = (int64_t)cnt[PMMG_HIT_BDY_STALE];
  out->nbdy_closest = (int64_t)cnt[PMMG_HIT_BDY_CLOSEST];
  out->steps_total = (int64_t)steps;
  out->stepmax = (int64_t)stepmax;
  out->wave_iters = (int64_t)cnt[kCntWaveIters];
  out->sorted = order[0] == 1;
  out->nvol_noseed = (int64_t)cnt[kCntNoSeed];
  out->nvol_stuck = (int64_t)cnt[kCntStuck];
  out->nvol_limit = (int64_t)cnt[kCntLimit];
  {
    int ad = 0;
    HIPCK(c, ctx_d2h(c, &ad, &((const Frame *)c->frame.p)->adaptive, sizeof(int)));
    out->seed_map_axes = ad;
    out->nbdy_fanscan = (int64_t)cnt[kCntFanScan];
  }
  float ms = 0.f;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[EV_START], c->ev[EV_PREP]));
  out->ms_prepare = ms;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[EV_SB0], c->ev[EV_ORDER]));
  out->ms_sort = ms; // on the second (and third) stream, concurrent with the seed grid
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[c->ev_vol0], c->ev[c->ev_vol]));
  out->ms_vol = ms;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[c->ev_vol0], c->ev[EV_WALK]));
  out->ms_vol_locate = ms;
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[EV_BDY0], c->ev[EV_BDY1]));
  out->ms_bdy = ms; // on the surface stream, concurrent with the volume kernels
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[c->ev_vol], c->ev[EV_JOIN]));
  out->ms_fallback = ms; // the volume queries' exhaustive search (the surface one is in ms_bdy)
  HIPCK(c, hipEventElapsedTime(&ms, c->ev[EV_START], c->ev[EV_END]));
  out->ms_total = ms;
  return 1;
}

int pmmg_hip_sync(pmmg_hip_ctx *c, pmmg_hip_stats *stats) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  for (pmmg_hip_ctx *l : c->lanes)
    if (hipStreamSynchronize(l->stream) != hipSuccess) {
      set_err(c, "sync: group lane failed: %s", l->err);
      return 0;
    }
  HIPCK(c, hipStreamSynchronize(c->stream));
  if (stats && c->pending) return collect_stats(c, stats);
  return 1;
}

int pmmg_hip_locate_interp(pmmg_hip_ctx *c, int np_new, const double *xyz_new, const uint8_t *pclass,
                           double *met_out, double *const *fields_out, int *elem_out, int8_t *hit_out,
                           pmmg_hip_stats *stats, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (c->bg.ne <= 0) {
    set_err(c, "locate_interp: no background set");
    return 0;
  }
  if (np_new <= 0) {
    if (stats) memset(stats, 0, sizeof(*stats));
    return 1;
  }
  if (!xyz_new || !pclass) {
    set_err(c, "locate_interp: xyz_new / pclass is NULL");
    return 0;
  }
  if (where == PMMG_HIP_DEVICE) {
    if (((uintptr_t)met_out & 15) && c->met_size == 6) {
      set_err(c, "locate_interp: a device tensor output must be 16-byte aligned");
      return 0;
    }
    if (!run_device(c, np_new, xyz_new, pclass, met_out, fields_out, elem_out, hit_out)) return 0;
    if (stats) return pmmg_hip_sync(c, stats);
    return 1;
  }
  // host mode: queries in, outputs out through the pinned staging buffers.
  // The device output rows start as a sentinel NaN, and only the rows the
  // step wrote (sentinel gone; elem / hit where hit != 0) are copied back, so
  // the caller's other rows stay untouched without being uploaded.
  size_t n = (size_t)np_new;
  const double t0 = now_s();
  if (!upload(c, c->h_xyz, xyz_new, sizeof(double) * 3 * n)) return 0;
  if (!upload(c, c->h_cls, pclass, n)) return 0;
  double *dmet = nullptr;
  auto sentinel_fill = [&](DevBuf &b, size_t ndbl) -> int {
    if (!ensure(c, b, sizeof(double) * ndbl)) return 0;
    hipLaunchKernelGGL(k_fill64, dim3(blocks_for((long long)ndbl, 4096)), dim3(kBlock), 0, c->stream,
                       (unsigned long long *)b.p, (long long)ndbl, kSentinel);
    return 1;
  };
  if (c->met_size) {
    if (!met_out) {
      set_err(c, "locate_interp: met_out is NULL");
      return 0;
    }
    if (!sentinel_fill(c->h_met, (size_t)c->met_size * n)) return 0;
    dmet = (double *)c->h_met.p;
  }
  c->h_f.resize(c->nfield);
  std::vector<double *> dfields(c->nfield > 0 ? c->nfield : 1, nullptr);
  for (int j = 0; j < c->nfield; j++) {
    if (!fields_out || !fields_out[j]) {
      set_err(c, "locate_interp: fields_out[%d] is NULL", j);
      return 0;
    }
    if (!sentinel_fill(c->h_f[j], (size_t)c->fsize[j] * n)) return 0;
    dfields[j] = (double *)c->h_f[j].p;
  }
  if (!ensure(c, c->h_elem, sizeof(int) * n) || !ensure(c, c->h_hit, n)) return 0;
  HIPCK(c, hipMemsetAsync(c->h_hit.p, 0, n, c->stream));
  if (!run_device(c, np_new, (const double *)c->h_xyz.p, (const uint8_t *)c->h_cls.p, dmet, dfields.data(),
                  (int *)c->h_elem.p, (int8_t *)c->h_hit.p))
    return 0;
  const double t1 = now_s();
  std::vector<int8_t> hh(n);
  if (!d2h_rows(c, hh.data(), c->h_hit.p, n, 1, AllRows{})) return 0;
  const double t2 = now_s();
  auto written = [&](size_t, const char *row) {
    unsigned long long u;
    memcpy(&u, row, 8);
    return u != kSentinel;
  };
  auto processed = [&](size_t r, const char *) { return hh[r] != 0; };
  if (dmet && !d2h_rows(c, met_out, dmet, n, sizeof(double) * c->met_size, written)) return 0;
  for (int j = 0; j < c->nfield; j++)
    if (!d2h_rows(c, fields_out[j], dfields[j], n, sizeof(double) * c->fsize[j], written)) return 0;
  if (elem_out && !d2h_rows(c, elem_out, c->h_elem.p, n, sizeof(int), processed)) return 0;
  if (hit_out)
    c->pool->run(n, n >= 65536 ? c->pool->th.size() + 1 : 1, [&](size_t a, size_t e) {
      for (size_t r = a; r < e; r++)
        if (hh[r]) hit_out[r] = hh[r];
    });
  if (c->verbose)
    fprintf(stderr, "[parmmg_hip] host locate: uploads + enqueue %.2f ms, step + hit codes %.2f ms, rows %.2f ms\n",
            1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (now_s() - t2));
  c->last_host_np = np_new; // what pmmg_hip_keep can keep
  c->last_host_met = c->met_size;
  c->last_host_fsize = c->fsize;
  if (stats) return collect_stats(c, stats);
  return 1;
}

int pmmg_hip_locate_interp_rec(pmmg_hip_ctx *c, int np_new, const double *xyz_new, const uint8_t *pclass,
                               double *rec_out, int *elem_out, int8_t *hit_out, pmmg_hip_stats *stats, int where) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (where != PMMG_HIP_DEVICE) {
    set_err(c, "locate_interp_rec: device pointers only (PMMG_HIP_DEVICE)");
    return 0;
  }
  if (c->bg.ne <= 0) {
    set_err(c, "locate_interp_rec: no background set");
    return 0;
  }
  if (!c->rec) {
    set_err(c, "locate_interp_rec: output records need packed input records (pmmg_hip_set_solutions_packed)");
    return 0;
  }
  if (np_new <= 0) {
    if (stats) memset(stats, 0, sizeof(*stats));
    return 1;
  }
  if (!xyz_new || !pclass || !rec_out || ((uintptr_t)rec_out & 15)) {
    set_err(c, "locate_interp_rec: xyz_new / pclass / rec_out NULL or rec_out not 16-byte aligned");
    return 0;
  }
  if (!run_device(c, np_new, xyz_new, pclass, nullptr, nullptr, elem_out, hit_out, rec_out)) return 0;
  if (stats) return pmmg_hip_sync(c, stats);
  return 1;
}

// ---- carry-over entry points (see "carry-over" above)

int pmmg_hip_keep(pmmg_hip_ctx *c, int slot) {
  if (!c) return 0;
  if (slot < 0 || slot >= 1024) {
    set_err(c, "keep: slot %d out of [0, 1024)", slot);
    return 0;
  }
  if (c->last_host_np <= 0) {
    set_err(c, "keep: no host-mode pmmg_hip_locate_interp to keep since the last keep");
    return 0;
  }
  if ((int)c->kept.size() <= slot) c->kept.resize(slot + 1);
  pmmg_hip_ctx::Kept &k = c->kept[slot];
  std::swap(k.xyz, c->h_xyz);
  k.met_size = c->last_host_met;
  if (k.met_size) std::swap(k.met, c->h_met);
  k.fsize = c->last_host_fsize;
  k.f.resize(k.fsize.size());
  for (size_t j = 0; j < k.f.size(); j++) std::swap(k.f[j], c->h_f[j]);
  k.np = c->last_host_np;
  k.valid = true;
  c->last_host_np = 0;
  return 1;
}

int pmmg_hip_carry_over(pmmg_hip_ctx *c, int slot, int np, const int *src) {
  if (!c) return 0;
  if (np == 0) { // drop the slot and free its device buffers
    if (c->carry_slot == slot && c->carry_bg) {
      set_err(c, "carry_over: slot %d is being carried (set_background took it, set_solutions has not run)", slot);
      return 0;
    }
    if (slot >= 0 && slot < (int)c->kept.size()) {
      pmmg_hip_ctx::Kept &k = c->kept[slot];
      HIPCK(c, hipSetDevice(c->device));
      if (!snap_join(c)) return 0;
      HIPCK(c, hipStreamSynchronize(c->stream));
      release(k.xyz);
      release(k.met);
      for (auto &b : k.f) release(b);
      k.f.clear();
      k.valid = false;
    }
    if (c->carry_slot == slot) carry_disarm(c);
    return 1;
  }
  if (slot < 0 || slot >= (int)c->kept.size() || !c->kept[slot].valid) {
    set_err(c, "carry_over: slot %d holds nothing (pmmg_hip_keep after a host-mode call)", slot);
    return 0;
  }
  const pmmg_hip_ctx::Kept &k = c->kept[slot];
  if (np <= 0 || (!src && np != k.np)) {
    set_err(c, "carry_over: %d vertices for %d kept points without a map", np, k.np);
    return 0;
  }
  c->carry_src.clear();
  if (src) {
    for (int i = 0; i < np; i++)
      if (src[i] < 0 || src[i] > k.np) {
        set_err(c, "carry_over: src[%d] = %d out of [0, %d]", i, src[i], k.np);
        return 0;
      }
    c->carry_src.assign(src, src + np);
  }
  c->carry_slot = slot;
  c->carry_np = np;
  c->carry_bg = false;
  return 1;
}

int pmmg_hip_release_scratch(pmmg_hip_ctx *c) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  HIPCK(c, hipStreamSynchronize(c->stream));
  HIPCK(c, hipStreamSynchronize(c->stream2));
  if (c->stream3) HIPCK(c, hipStreamSynchronize(c->stream3));
  pmmg_snap_cache_free(&c->snap_cache);
  for (DevBuf *b : {&c->bvals2, &c->rs_hist, &c->rs_csum}) release(*b);
  for (pmmg_hip_ctx *l : c->lanes) pmmg_hip_destroy(l);
  c->lanes.clear();
  return 1;
}

int64_t pmmg_hip_bytes_up(pmmg_hip_ctx *c, int reset) {
  if (!c) return -1;
  const int64_t b = c->bytes_up;
  if (reset) c->bytes_up = 0;
  return b;
}

// ---- many groups in one call

static void stats_sum(pmmg_hip_stats *a, const pmmg_hip_stats &b) {
  a->nvol += b.nvol; a->nbdy += b.nbdy;
  a->nvol_walk += b.nvol_walk; a->nvol_exhaust += b.nvol_exhaust; a->nvol_closest += b.nvol_closest;
  a->nvol_exact += b.nvol_exact;
  a->nbdy_face += b.nbdy_face; a->nbdy_edge += b.nbdy_edge; a->nbdy_vertex += b.nbdy_vertex;
  a->nbdy_wedge += b.nbdy_wedge; a->nbdy_cone += b.nbdy_cone; a->nbdy_exhaust += b.nbdy_exhaust;
  a->nbdy_stale += b.nbdy_stale; a->nbdy_closest += b.nbdy_closest;
  a->steps_total += b.steps_total; a->wave_iters += b.wave_iters;
  a->sorted += b.sorted; // the number of groups whose queries were Morton-binned
  if (b.stepmax > a->stepmax) a->stepmax = b.stepmax;
  a->ms_prepare += b.ms_prepare; a->ms_sort += b.ms_sort; a->ms_vol += b.ms_vol; a->ms_bdy += b.ms_bdy;
  a->ms_fallback += b.ms_fallback; a->ms_total += b.ms_total; a->ms_vol_locate += b.ms_vol_locate;
  a->nvol_noseed += b.nvol_noseed; a->nvol_stuck += b.nvol_stuck; a->nvol_limit += b.nvol_limit;
  a->seed_map_axes |= b.seed_map_axes;
  a->nbdy_fanscan += b.nbdy_fanscan;
}

static pmmg_hip_ctx *group_lane(pmmg_hip_ctx *c, int j) {
  while ((int)c->lanes.size() <= j) {
    const bool first = c->lanes.empty();
    pmmg_hip_ctx *l = create_ctx(c->device, c->options, false, first && c->lane0 ? c : nullptr);
    if (!l) {
      set_err(c, "locate_interp_groups: cannot create group lane %d", (int)c->lanes.size());
      return nullptr;
    }
    if (c->lane_streams == 1 && !l->borrowed_streams) {
      (void)hipStreamDestroy(l->stream2);
      l->stream2 = l->stream;
    }
#ifdef PMMG_HIP_MEASURE
    if (c->lane_streams == 3 && !l->borrowed_streams) { // both of a lane's streams at the highest priority
      int lo = 0, hi = 0;
      (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
      (void)hipStreamDestroy(l->stream);
      (void)hipStreamDestroy(l->stream2);
      (void)hipStreamCreateWithPriority(&l->stream, hipStreamNonBlocking, hi);
      (void)hipStreamCreateWithPriority(&l->stream2, hipStreamNonBlocking, hi);
    }
#endif
    c->lanes.push_back(l);
  }
  return c->lanes[j];
}

// one lane's share of a groups call: groups j, j + L, j + 2L, ... enqueued in
// order (each waited for and its counters summed when stats are wanted)
static int lane_groups(pmmg_hip_ctx *l, int j, int L, int ngroup, const pmmg_hip_group *groups, bool want,
                       pmmg_hip_stats *sum, int *bad) {
  if (hipSetDevice(l->device) != hipSuccess) {
    *bad = j;
    return 0;
  }
  for (int i = j; i < ngroup; i += L) {
    const pmmg_hip_group &g = groups[i];
    const int ok =
        (g.tet8 ? set_background_impl(l, g.np, g.xyz, g.ne, nullptr, nullptr, g.tet8, g.nt, g.triv, g.adjt, g.hausd,
                                      PMMG_HIP_DEVICE)
                : (g.tetv && set_background_impl(l, g.np, g.xyz, g.ne, g.tetv, g.adja, nullptr, g.nt, g.triv, g.adjt,
                                                 g.hausd, PMMG_HIP_DEVICE))) &&
        pmmg_hip_set_solutions(l, g.met_size, g.met, g.nfield, g.field_size, g.fields, PMMG_HIP_DEVICE) &&
        pmmg_hip_locate_interp(l, g.np_new, g.xyz_new, g.pclass, g.met_out, g.fields_out, g.elem_out, g.hit_out,
                               nullptr, PMMG_HIP_DEVICE);
    pmmg_hip_stats st;
    if (!ok || (want && (hipStreamSynchronize(l->stream) != hipSuccess || !collect_stats(l, &st)))) {
      *bad = i;
      return 0;
    }
    if (want) stats_sum(sum, st);
  }
  return 1;
}

int pmmg_hip_locate_interp_groups(pmmg_hip_ctx *c, int ngroup, const pmmg_hip_group *groups,
                                  pmmg_hip_stats *stats) {
  if (!c) return 0;
  if (stats) memset(stats, 0, sizeof(*stats));
  if (ngroup <= 0) return 1;
  if (!groups) {
    set_err(c, "locate_interp_groups: groups is NULL");
    return 0;
  }
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (c->stream2_hi) { // (see run_device)
    HIPCK(c, hipStreamSynchronize(c->stream2_hi));
    HIPCK(c, hipStreamDestroy(c->stream2_hi));
    c->stream2_hi = nullptr;
  }
  // a large call's extra streams (binning, refill) are released before the lanes take theirs, so that the
  // lanes' streams find the queues those held (a later large call creates them again)
  for (hipStream_t *x : {&c->stream3, &c->stream_f})
    if (*x && c->lanes.size() < (size_t)std::min(c->group_lanes, ngroup)) {
      HIPCK(c, hipStreamSynchronize(*x));
      HIPCK(c, hipStreamDestroy(*x));
      *x = nullptr;
    }
  // lanes dealt an equal number of groups: ceil(n / rounds) lanes for the rounds the most lanes need
  // (10 groups, 5 lanes: 2 each; 7 groups: 4 lanes of 2, 2, 2, 1 rather than 5 of 2, 2, 1, 1, 1)
  const int Lmax = std::max(1, c->group_lanes), rounds = (ngroup + Lmax - 1) / Lmax;
  const int L = std::max(1, std::min(ngroup, (ngroup + rounds - 1) / rounds));
  std::vector<pmmg_hip_ctx *> lane(L);
  for (int j = 0; j < L; j++)
    if (!(lane[j] = group_lane(c, j))) return 0;
  // every lane enqueues its groups from its own host thread (the enqueue of
  // ~25 launches per group is the host's share of a small group)
  std::vector<pmmg_hip_stats> sums(L);
  std::vector<int> bad(L, -1), ok(L, 1);
  for (auto &x : sums) memset(&x, 0, sizeof(x));
  if (L > 1 && !c->lane_pool) c->lane_pool = new Pool(c->group_lanes - 1);
  auto work = [&](size_t a, size_t e) {
    for (size_t j = a; j < e; j++)
      ok[j] = lane_groups(lane[j], (int)j, L, ngroup, groups, stats != nullptr, &sums[j], &bad[j]);
  };
  if (L > 1) c->lane_pool->run((size_t)L, (size_t)L, work);
  else work(0, 1);
  HIPCK(c, hipSetDevice(c->device));
  int first = -1, fl = 0;
  for (int j = 0; j < L; j++)
    if (!ok[j] && (first < 0 || bad[j] < first)) {
      first = bad[j];
      fl = j;
    }
  if (first >= 0) {
    const std::string why = lane[fl]->err;
    set_err(c, "locate_interp_groups: group %d: %s", first, why.c_str());
    return 0;
  }
  if (stats)
    for (int j = 0; j < L; j++) stats_sum(stats, sums[j]);
  return 1;
}

// ---- background snapshot (pmmg_snapshot.hip)

static bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

int pmmg_hip_build_adjacency(pmmg_hip_ctx *c, int np, int ne, const int *tetv, int *adja, int *tet8) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (np <= 0 || ne <= 0 || !tetv || (!adja && !tet8)) {
    set_err(c, "build_adjacency: invalid arguments (np=%d ne=%d)", np, ne);
    return 0;
  }
  if (ne >= (1 << 29)) {
    set_err(c, "build_adjacency: %d tetra exceed the 4*k+i adjacency encoding (2^29)", ne);
    return 0;
  }
  if (!aligned16(tetv) || (adja && !aligned16(adja)) || (tet8 && !aligned16(tet8))) {
    set_err(c, "build_adjacency: device arrays must be 16-byte aligned");
    return 0;
  }
  return pmmg_snap_adjacency(c->stream, np, ne, tetv, adja, tet8, &c->snap_cache, c->err, sizeof(c->err));
}

int pmmg_hip_tetra_qual(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tetv, int met_size,
                        const double *met, double *qual, double *minqual) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (np < 0 || ne < 0 || (ne > 0 && (!xyz || !tetv || !qual)) || !minqual ||
      (met_size == 6 && ne > 0 && !met) || (met_size != 0 && met_size != 1 && met_size != 6)) {
    set_err(c, "tetra_qual: invalid arguments (np=%d ne=%d met_size=%d)", np, ne, met_size);
    return 0;
  }
  if (ne > 0 && !aligned16(tetv)) {
    set_err(c, "tetra_qual: tetv must be 16-byte aligned");
    return 0;
  }
  if (!ensure(c, c->qmin, sizeof(unsigned long long))) return 0;
  unsigned long long bits = 0;
  if (!pmmg_qual_tetra(c->stream, np, xyz, ne, tetv, met_size, met, qual, (unsigned long long *)c->qmin.p, &bits)) {
    set_err(c, "tetra_qual: kernel launch or copy failed");
    return 0;
  }
  // MMG3D_tetraQual: minqual starts at 2/ALPHAD, returns ALPHAD * minqual
  const double alphad = 20.7846096908265; // MMG3D_ALPHAD = 12 sqrt(3): a regular tetra has quality 1
  double mn = 2.0 / alphad;
  if (bits != ~0ULL) {
    double q;
    memcpy(&q, &bits, sizeof q);
    if (q < mn) mn = q;
  }
  *minqual = alphad * mn;
  return 1;
}

int pmmg_hip_compute_wgt_mesh(pmmg_hip_ctx *c, int np, const double *xyz, int ne, const int *tetv, const int *xt,
                              const uint16_t *ftag, int met_size, const double *met, int tag, double *qual) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (np < 0 || ne < 0 || (ne > 0 && (!xyz || !tetv || !xt || !ftag || !qual)) ||
      (met_size != 0 && met_size != 1 && met_size != 6) || (met_size && ne > 0 && !met)) {
    set_err(c, "compute_wgt_mesh: invalid arguments (np=%d ne=%d met_size=%d)", np, ne, met_size);
    return 0;
  }
  if (ne > 0 && (!aligned16(tetv) || ((uintptr_t)ftag & 7))) {
    set_err(c, "compute_wgt_mesh: tetv must be 16-byte and ftag 8-byte aligned");
    return 0;
  }
  if (!pmmg_wgt_mesh(c->stream, xyz, ne, tetv, xt, ftag, met_size, met, tag, qual)) {
    set_err(c, "compute_wgt_mesh: kernel launch failed");
    return 0;
  }
  return 1;
}

int pmmg_hip_compute_wgt_faces(pmmg_hip_ctx *c, int np, const double *xyz, const int *tetv, int nface,
                               const int *face, int met_size, const double *met, double *wgt) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (np < 0 || nface < 0 || (nface > 0 && (!xyz || !tetv || !face || !wgt)) ||
      (met_size != 0 && met_size != 1 && met_size != 6) || (met_size && nface > 0 && !met)) {
    set_err(c, "compute_wgt_faces: invalid arguments (np=%d nface=%d met_size=%d)", np, nface, met_size);
    return 0;
  }
  if (nface > 0 && (!aligned16(tetv) || ((uintptr_t)face & 7))) {
    set_err(c, "compute_wgt_faces: tetv must be 16-byte and face 8-byte aligned");
    return 0;
  }
  if (!pmmg_wgt_faces(c->stream, xyz, tetv, nface, face, met_size, met, wgt)) {
    set_err(c, "compute_wgt_faces: kernel launch failed");
    return 0;
  }
  return 1;
}

int pmmg_hip_build_boundary(pmmg_hip_ctx *c, int np, int ne, const int *tet8, const int *tetv, const int *adja,
                            const int *tref, int cap, int *nt, int *triv, int *adjt) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  const bool packed = tet8 != nullptr;
  if (np <= 0 || ne <= 0 || !nt || (!packed && (!tetv || !adja)) || cap < 0 || (cap > 0 && !triv)) {
    set_err(c, "build_boundary: invalid arguments (np=%d ne=%d cap=%d)", np, ne, cap);
    return 0;
  }
  const int *t0 = packed ? tet8 : tetv, *a0 = packed ? tet8 + 4 : adja;
  if (!aligned16(t0) || !aligned16(a0)) {
    set_err(c, "build_boundary: device tetra arrays must be 16-byte aligned");
    return 0;
  }
  return pmmg_snap_boundary(c->stream, np, ne, t0, packed ? 2 : 1, a0, packed ? 2 : 1, tref, cap, nt, triv, adjt,
                            &c->snap_cache, c->err, sizeof(c->err));
}

void *pmmg_hip_malloc(pmmg_hip_ctx *c, int64_t bytes) {
  if (!c || bytes < 0) return nullptr;
  if (hipSetDevice(c->device) != hipSuccess) return nullptr;
  void *p = nullptr;
  if (hipMalloc(&p, bytes > 0 ? (size_t)bytes : 16) != hipSuccess) {
    set_err(c, "hipMalloc(%lld) failed", (long long)bytes);
    return nullptr;
  }
  return p;
}

int pmmg_hip_free(pmmg_hip_ctx *c, void *p) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  HIPCK(c, hipFree(p));
  return 1;
}

int pmmg_hip_memcpy_h2d(pmmg_hip_ctx *c, void *dst, const void *src, int64_t bytes) {
  if (!c || bytes < 0) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (!h2d(c, dst, src, (size_t)bytes, c->stream)) return 0;
  HIPCK(c, hipStreamSynchronize(c->stream));
  return 1;
}

// ---- the split of a group over the node's GPUs (pmmg_comm.hpp)

int pmmg_hip_comm_unique_id(void *id) {
  if (!id) return 0;
  Rccl &R = rccl();
  if (!R.ok) {
    fprintf(stderr, "[parmmg_hip] comm_unique_id: %s\n", R.why);
    return 0;
  }
  ncclUniqueId u;
  const ncclResult_t e = R.getUniqueId(&u);
  if (e != ncclSuccess) {
    fprintf(stderr, "[parmmg_hip] ncclGetUniqueId: %s\n", R.errorString(e));
    return 0;
  }
  memcpy(id, &u, sizeof(u));
  return 1;
}

static void comm_release(pmmg_hip_ctx *c) {
  if (c->comm && c->comm_owned && rccl().ok) (void)rccl().commDestroy(c->comm);
  c->comm = nullptr;
  c->comm_owned = false;
  c->comm_rank = c->comm_size = 0;
}

static constexpr int kAgView = 8; // int64 per rank in the all-gather's agreement (ag_agree)

int pmmg_hip_comm_init(pmmg_hip_ctx *c, int nranks, int rank, const void *id) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (nranks < 1 || rank < 0 || rank >= nranks || !id) {
    set_err(c, "comm_init: invalid arguments (nranks=%d rank=%d)", nranks, rank);
    return 0;
  }
  Rccl &R = rccl();
  if (!R.ok) {
    set_err(c, "comm_init: %s", R.why);
    return 0;
  }
  comm_release(c);
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t comm = nullptr;
  const ncclResult_t e = R.commInitRank(&comm, nranks, u, rank);
  if (e != ncclSuccess) {
    set_err(c, "ncclCommInitRank(%d of %d): %s", rank, nranks, R.errorString(e));
    return 0;
  }
  c->comm = comm;
  c->comm_owned = true;
  c->comm_rank = rank;
  c->comm_size = nranks;
  // the all-gather's agreement buffer, allocated here so that pmmg_hip_allgather_points allocates nothing
  // before every rank has agreed (ag_agree)
  return ensure(c, c->ag_chk, sizeof(long long) * kAgView * (nranks + 1));
}

int pmmg_hip_comm_attach(pmmg_hip_ctx *c, void *comm, int nranks, int rank) {
  if (!c) return 0;
  if (nranks < 1 || rank < 0 || rank >= nranks || !comm) {
    set_err(c, "comm_attach: invalid arguments (nranks=%d rank=%d)", nranks, rank);
    return 0;
  }
  if (!rccl().ok) {
    set_err(c, "comm_attach: %s", rccl().why);
    return 0;
  }
  comm_release(c);
  c->comm = (ncclComm_t)comm;
  c->comm_owned = false;
  c->comm_rank = rank;
  c->comm_size = nranks;
  return ensure(c, c->ag_chk, sizeof(long long) * kAgView * (nranks + 1)); // (see pmmg_hip_comm_init)
}

// The all-gather's agreement: every rank that holds a
// communicator takes part in one small all-gather of its view of the call —
// {local arguments valid and buffers allocated, K, nslot, the slot sizes, elem
// / hit given, a hash of counts[]} — before the data collective, and every
// rank then takes the same decision: either all gather, or all return 0 (a
// rank that returned early used to leave the others inside ncclAllGather, and
// records of different sizes R = 8 K + 8 were undefined behaviour).
static int ag_agree(pmmg_hip_ctx *c, const long long *mine, std::vector<long long> &all) {
  const int N = c->comm_size;
  all.assign((size_t)kAgView * N, 0);
  if (!ensure(c, c->ag_chk, sizeof(long long) * kAgView * (N + 1))) return 0;
  long long *d = (long long *)c->ag_chk.p;
  hipStream_t s = c->stream;
  HIPCK(c, hipMemcpyAsync(d, mine, sizeof(long long) * kAgView, hipMemcpyHostToDevice, s));
  const ncclResult_t e = rccl().allGather(d, d + kAgView, kAgView, ncclInt64, c->comm, s);
  if (e != ncclSuccess) {
    set_err(c, "ncclAllGather (agreement): %s", rccl().errorString(e));
    return 0;
  }
  HIPCK(c, hipMemcpyAsync(all.data(), d + kAgView, sizeof(long long) * kAgView * N, hipMemcpyDeviceToHost, s));
  HIPCK(c, hipStreamSynchronize(s));
  return 1;
}

int pmmg_hip_allgather_points(pmmg_hip_ctx *c, const int64_t *counts, int nslot, const int *slot_size,
                              const double *const *rows, double *const *rows_all, const int *elem, int *elem_all,
                              const int8_t *hit, int8_t *hit_all) {
  if (!c) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if (!c->comm) {
    set_err(c, "allgather_points: no communicator (pmmg_hip_comm_init / pmmg_hip_comm_attach)");
    return 0;
  }
  const int N = c->comm_size;
  // local checks: a failure is recorded (ok = 0), not returned, so that this
  // rank still takes part in the agreement below
  bool ok = true;
  char why[256] = {0};
  if (!counts || nslot < 0 || nslot > kMaxSlot || (nslot > 0 && (!slot_size || !rows || !rows_all)) ||
      (!elem) != (!elem_all) || (!hit) != (!hit_all)) {
    snprintf(why, sizeof(why), "allgather_points: invalid arguments (nslot=%d)", nslot);
    ok = false;
  }
  AgSlots S{};
  long long sizes_code = 0;
  if (ok) {
    S.n = nslot;
    for (int j = 0; j < nslot && ok; j++) {
      if (slot_size[j] < 1 || slot_size[j] > 6 || !rows_all[j] || (counts[c->comm_rank] > 0 && !rows[j])) {
        snprintf(why, sizeof(why), "allgather_points: slot %d (size %d) invalid", j, slot_size[j]);
        ok = false;
        break;
      }
      S.in[j] = rows[j];
      S.out[j] = rows_all[j];
      S.size[j] = slot_size[j];
      S.K += slot_size[j];
      sizes_code = sizes_code * 8 + slot_size[j];
    }
  }
  std::vector<long long> off((size_t)N + 1, 0);
  long long maxn = 0;
  unsigned long long chash = 0x9E3779B97F4A7C15ULL;
  for (int r = 0; r < N && ok; r++) {
    if (counts[r] < 0) {
      snprintf(why, sizeof(why), "allgather_points: counts[%d] = %lld", r, (long long)counts[r]);
      ok = false;
      break;
    }
    off[r + 1] = off[r] + counts[r];
    maxn = std::max(maxn, (long long)counts[r]);
    chash = (chash ^ (unsigned long long)counts[r]) * 0x100000001B3ULL;
  }
  const long long R = 8LL * S.K + 8;
  if (ok && maxn > 0 &&
      (!ensure(c, c->ag_send, (size_t)(R * maxn)) || !ensure(c, c->ag_recv, (size_t)(R * maxn * N)) ||
       !ensure(c, c->ag_off, sizeof(long long) * off.size()))) {
    snprintf(why, sizeof(why), "allgather_points: buffers: %s", c->err);
    ok = false;
  }
  // the arguments that must be identical on every rank: nslot, slot_size[],
  // whether elem / hit are given, counts[] (hence K, R and maxn)
  const long long mine[kAgView] = {ok ? 1 : 0, S.K, nslot, sizes_code, elem ? 1 : 0, hit ? 1 : 0,
                                   (long long)(chash >> 1), maxn};
  std::vector<long long> all;
  if (!ag_agree(c, mine, all)) return 0;
  if (!ok) {
    set_err(c, "%s", why);
    return 0;
  }
  for (int r = 0; r < N; r++) {
    const long long *v = &all[(size_t)kAgView * r];
    if (!v[0]) {
      set_err(c, "allgather_points: rank %d's arguments are invalid", r);
      return 0;
    }
    for (int j = 1; j < kAgView; j++)
      if (v[j] != all[j]) {
        set_err(c, "allgather_points: rank %d disagrees with rank 0 on %s", r,
                j <= 3 ? "the slot layout" : (j <= 5 ? "elem / hit" : "counts[]"));
        return 0;
      }
  }
  const long long n = counts[c->comm_rank];
  if (maxn == 0) return 1;
  hipStream_t s = c->stream;
  HIPCK(c, hipMemcpyAsync(c->ag_off.p, off.data(), sizeof(long long) * off.size(), hipMemcpyHostToDevice, s));
  if (n > 0)
    hipLaunchKernelGGL(k_ag_pack, dim3(blocks_for(n, 4096)), dim3(kBlock), 0, s, S, elem, hit, n, (char *)c->ag_send.p);
  HIPCK(c, hipGetLastError());
  const ncclResult_t e =
      rccl().allGather(c->ag_send.p, c->ag_recv.p, (size_t)(R * maxn), ncclInt8, c->comm, s);
  if (e != ncclSuccess) {
    set_err(c, "ncclAllGather: %s", rccl().errorString(e));
    return 0;
  }
  hipLaunchKernelGGL(k_ag_unpack, dim3(blocks_for(off[N], 8192)), dim3(kBlock), 0, s, S, (const char *)c->ag_recv.p,
                     maxn, N, (const long long *)c->ag_off.p, elem_all, hit_all);
  HIPCK(c, hipGetLastError());
  HIPCK(c, hipStreamSynchronize(s));
  return 1;
}

int pmmg_hip_memcpy_d2h(pmmg_hip_ctx *c, void *dst, const void *src, int64_t bytes) {
  if (!c || bytes < 0) return 0;
  HIPCK(c, hipSetDevice(c->device));
  if (!snap_join(c)) return 0;
  if ((size_t)bytes < kStageMin) {
    HIPCK(c, hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCK(c, hipStreamSynchronize(c->stream));
    return 1;
  }
  return d2h_rows(c, dst, src, (size_t)bytes, 1, AllRows{});
}

} // extern "C"
