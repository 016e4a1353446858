# Round 5: persistent-kernel phase stamps (diagnostic build tools/_diag, scripts/build_probes.sh) for the
# headline (n = 2e6), one rank of 8 (2.5e5) and config 2's run starts (47 279), plain and guarded kernels
set -o pipefail
mkdir -p gpurun_out/r05st
for n in 2000000 250000 47279; do
  for gd in 0 1; do
    PROBE_GUARD=$gd timeout -k 10 120 tools/_diag/probe_stamps $n p > gpurun_out/r05st/stamps_n${n}_guard${gd}.log 2>&1 || exit 1
    grep -E "^stamps|^sweep|^compute|winner" gpurun_out/r05st/stamps_n${n}_guard${gd}.log | sed "s/^/n=$n guard=$gd  /"
  done
done
