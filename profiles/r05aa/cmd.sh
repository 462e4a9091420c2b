set -o pipefail
mkdir -p gpurun_out/r05aa
for v in "none" "cfg3 off" "cfg3 auto" "cfg3 on" "cfg2 on"; do
  timeout -k 10 300 python3 -u tools/groups_after_big.py $v > gpurun_out/r05aa/"${v// /_}".log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/r05aa/${v// /_}.log)"
done
