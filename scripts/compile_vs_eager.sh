#!/bin/bash
# torch.compile vs eager for the model sizes of the reference sweep (benchmark.py:262-304 protocol via
# cs336_systems.bench.e2e), bf16 autocast, one process per (size, mode).
#   bash scripts/compile_vs_eager.sh [ctx] [sizes...]   (GPU box; JSON per run in gpurun_out/cve/)
set -o pipefail
ctx=${1:-512}; shift; sizes=${@:-small medium large xl 2.7b}
O=gpurun_out/cve; mkdir -p $O
# heartbeat: Inductor's first compile (Triton JIT of the few non-custom-op kernels) prints nothing
( while sleep 60; do echo "[heartbeat $(date +%T)]"; done ) &
HB=$!; trap "kill $HB" EXIT
for s in $sizes; do
  for m in eager compile; do
    flag=""; [ $m = compile ] && flag="--compile"
    timeout -k 10 600 python -u -m cs336_systems.bench.e2e --sizes $s --ctx $ctx --mixed $flag --json $O/${s}_$m.json \
      > $O/${s}_$m.log 2>&1 || { echo "$s $m failed: $?"; tail -5 $O/${s}_$m.log; exit 1; }
    python - "$O/${s}_$m.json" <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))[0]
print(f"{r['size']:6s} compile={r['compile']!s:5s} fwd {r['fwd_ms']:.2f} bwd {r['bwd_ms']:.2f} step {r['step_ms']:.2f} ms", flush=True)
PY
  done
done
