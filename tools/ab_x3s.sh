set -u
for v in d2 d3 default; do
  if [ $v = default ]; then
    timeout -k 10 200 python -u tools/x3s_ab.py > gpurun_out/x3s_ab_$v.jsonl 2> gpurun_out/x3s_ab_$v.err || exit 1
  else
    RQVAE_HIP_LIB=build_ab/$v.so timeout -k 10 200 python -u tools/x3s_ab.py > gpurun_out/x3s_ab_$v.jsonl 2> gpurun_out/x3s_ab_$v.err || exit 1
  fi
done
timeout -k 10 300 python -u -m pytest tests/test_gemm_x3s_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/x3s_tests.log 2>&1
tail -15 gpurun_out/x3s_tests.log
