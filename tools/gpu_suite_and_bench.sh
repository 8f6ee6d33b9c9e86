#!/usr/bin/env bash
# GPU suite, smoke, then the headline bench (bench.py defaults): gpurun_out/suite/{pytest.log,smoke.log,bench.json}
set -o pipefail
mkdir -p gpurun_out/suite
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite/pytest.log 2>&1 || { tail -40 gpurun_out/suite/pytest.log; exit 1; }
tail -2 gpurun_out/suite/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1 || { tail -20 gpurun_out/suite/smoke.log; exit 1; }
tail -2 gpurun_out/suite/smoke.log
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 900 python3 bench.py --json-out gpurun_out/suite/bench.json > gpurun_out/suite/bench.log 2>&1 || { tail -20 gpurun_out/suite/bench.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/suite/bench.json'))
print('value', d['value'], 'ttft', d['ttft_ms'], 'decode', d['decode_ms_per_token'])
print('lat', [p['decode_ms_per_token'] for p in d['latency_points']['points']])
print('proxy', [p['decode_ms_per_token'] for p in d['tp_rank_proxy']['points']])
print('mp1', d.get('mp1_point', {}).get('point', {}).get('decode_ms_per_token'))
print('ttft2048', d.get('ttft'))
print('cal', d.get('calibration'))
"
fi
