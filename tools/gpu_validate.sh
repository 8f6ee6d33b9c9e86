set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v_gputests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/v_gputests.log; exit 1; }
tail -3 gpurun_out/v_gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v_smoke.log 2>&1 && tail -1 gpurun_out/v_smoke.log
timeout -k 10 420 python -u bench.py > gpurun_out/v_bench.log 2>&1; echo bench rc=$?; tail -2 gpurun_out/v_bench.log
