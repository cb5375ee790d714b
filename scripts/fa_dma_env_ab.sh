#!/bin/bash
# CS336_FA_DMA=1 (LDS-DMA forward everywhere) vs the default selection, same box, two rounds
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python scripts/fa_ab.py > gpurun_out/fa_env_def_$r.jsonl 2>&1 || exit 1
  CS336_FA_DMA=1 timeout -k 10 200 python scripts/fa_ab.py > gpurun_out/fa_env_dma1_$r.jsonl 2>&1 || exit 1
done
python - <<'P'
import json
for r in (1,2):
  b=[json.loads(l) for l in open(f'gpurun_out/fa_env_def_{r}.jsonl') if l.startswith('{')]
  n=[json.loads(l) for l in open(f'gpurun_out/fa_env_dma1_{r}.jsonl') if l.startswith('{')]
  for x,y in zip(b,n):
    print(r, x['B'],x['H'],x['N'],x['D'],x['causal'],'fwd',x['fwd_tflops'],'->',y['fwd_tflops'],'bwd',x['bwd_tflops'],y['bwd_tflops'])
P
