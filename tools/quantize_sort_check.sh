set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_tokenizer_kmeans_gpu.py tests/test_quantize_gpu.py tests/test_fused_decoder_gpu.py tests/test_reference_fixtures_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/qtests.log" 2>&1 || { tail -30 "$O/qtests.log"; exit 1; }
tail -1 "$O/qtests.log"
bash tools/prof_rq.sh > /dev/null && python3 tools/trace_shapes.py "$O/prof/rqonly_kernel_trace.csv" sort_
