#!/bin/bash
# Rehearsal of the driver's N=4 and N=8 bench commands on ONE GPU (all ranks share the card, so
# the transport chain is ipc -> host; the numbers are not a scaling measurement).
set -o pipefail
mkdir -p gpurun_out
export HEAT2D_NO_BUILD=1
for n in 4 8; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29700 + n)) bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/rehearse_n$n.json 2> gpurun_out/rehearse_n$n.err || { echo "N=$n failed"; tail -20 gpurun_out/rehearse_n$n.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/rehearse_n$n.json') if l.startswith('{')][-1]); print('N=$n', d['config']['transport'], d['config']['pipeline'], '%.3e' % d['value'], 'verified', d['verified'], 'gate', [(g['transport'], g['ok']) for g in d['gate']])"
done
