# Round 6, after the bounds slots and the streamed sums in LDS under the guard: phase stamps of the headline
# shape (n = 2e6) guarded and unguarded, and of config 2's all-row shape (2e5), diagnostic build ab/diag
set -o pipefail
mkdir -p gpurun_out/r06st2
run() {  # name, env..., n
  local name=$1; shift
  timeout -k 10 120 env "$@" > gpurun_out/r06st2/$name.log 2>&1 || { echo "FAIL $name"; tail -3 gpurun_out/r06st2/$name.log; exit 1; }
  grep -E "^stamps|^sweep:|^guard|^compute split|^publish split" gpurun_out/r06st2/$name.log | sed "s/^/$name  /"
}
run n2000000_g0 PROBE_GUARD=0 ab/diag/probe_stamps 2000000 p
run n2000000_g1 PROBE_GUARD=1 ab/diag/probe_stamps 2000000 p
run n200000_g0 PROBE_GUARD=0 ab/diag/probe_stamps 200000 p
run n200000_g1 PROBE_GUARD=1 ab/diag/probe_stamps 200000 p
