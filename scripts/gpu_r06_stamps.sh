# Round 6: persistent-kernel phase stamps (diagnostic build ab/diag, scripts/build_probes.sh): the headline
# (n = 2e6; guarded plan 8 register rows, unguarded 9 and 8), one rank of 8 (2.5e5), config 2's run starts
# (47 279) and the LV call's run starts (118 015) -- unguarded and guarded
set -o pipefail
mkdir -p gpurun_out/r06st
run() {  # name, env..., n
  local name=$1; shift
  timeout -k 10 120 env "$@" > gpurun_out/r06st/$name.log 2>&1 || { echo "FAIL $name"; tail -3 gpurun_out/r06st/$name.log; exit 1; }
  grep -E "^stamps|^sweep|^guard|^compute split|^publish split" gpurun_out/r06st/$name.log | sed "s/^/$name  /"
}
for n in 2000000 250000 47279 118015; do
  run n${n}_g0 PROBE_GUARD=0 ab/diag/probe_stamps $n p
  run n${n}_g1 PROBE_GUARD=1 ab/diag/probe_stamps $n p
done
run n2000000_g0_rt8 PROBE_GUARD=0 PROBE_CMP=8 ab/diag/probe_stamps 2000000 p
