set -o pipefail
for c in 308c1a3 7b5067c 48ce47d; do
  (cd _ab/$c && timeout -k 10 300 python3 -u tools/groups_only.py --no-parity > ../../gpurun_out/r05i_$c.log 2>&1) || exit 1
  tail -1 gpurun_out/r05i_$c.log
done
timeout -k 10 300 python3 -u tools/groups_only.py --no-parity > gpurun_out/r05i_head.log 2>&1 && tail -1 gpurun_out/r05i_head.log
