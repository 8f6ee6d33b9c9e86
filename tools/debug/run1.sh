set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm4_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 | tee gpurun_out/g4_tests2.log
B="timeout -k 10 200 python -u tools/bench_gemm.py"
$B --ops gate_up --mode swiglu --rms --m 2048 4096 --tile 1 7 --rounds 2 | tee gpurun_out/g4_epi2.jsonl
$B --ops qkv --rms --m 2048 4096 --tile 1 7 --rounds 2 --no-blas | tee -a gpurun_out/g4_epi2.jsonl
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I jax_llama_amd/csrc/kernels tools/debug/gemm4w_probe.hip -o /tmp/gemm4w_probe
timeout -k 10 60 /tmp/gemm4w_probe 1000 2560 1024 3 1 14 | tee -a gpurun_out/g4_ring.jsonl
timeout -k 10 60 /tmp/gemm4w_probe 700 1280 4096 3 1 14 | tee -a gpurun_out/g4_ring.jsonl
for s in "4096 28672 4096" "32768 6144 4096" "2048 28672 4096" "32768 4096 14336"; do
timeout -k 10 120 /tmp/gemm4w_probe $s 10 1 -5 | tee -a gpurun_out/g4_ring.jsonl
done
