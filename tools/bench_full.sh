#!/usr/bin/env bash
# The driver's headline run (bench.py defaults) with the tuner's picks written to gpurun_out/tune/ (JLA_TUNE_FILE), so
# the measured plans can be committed as the packaged table (jax_llama_amd/ops/tune_gfx950.json). Output: gpurun_out/full/.
set -o pipefail
mkdir -p gpurun_out/full gpurun_out/tune
export JLA_TUNE_FILE=${JLA_TUNE_FILE:-$PWD/gpurun_out/tune/tune_gfx950.json}
timeout -k 10 1100 python3 -u bench.py ${EXTRA:-} --json-out gpurun_out/full/bench.json > gpurun_out/full/bench.log 2>&1
rc=$?
python3 -c "
import json; d=json.load(open('gpurun_out/full/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'ttft', d['ttft_ms'], 'decode', d['decode_ms_per_token'])
print('lat', [p['decode_ms_per_token'] for p in d['latency_points']['points']])
print('proxy', [p['decode_ms_per_token'] for p in d['tp_rank_proxy']['points']])
print('mp1', d.get('mp1_point', {}).get('point', {}).get('decode_ms_per_token'))
print('ttft2048', d.get('ttft', {}).get('ttft_ms'), 'sampled', d.get('sampled', {}).get('tokens_per_sec'))
print('cal', d.get('calibration'))
" || tail -20 gpurun_out/full/bench.log
exit $rc
