set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_quantize_gpu.py tests/test_tokenizer_kmeans_gpu.py tests/test_reference_fixtures_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/utests.log" 2>&1 || { tail -30 "$O/utests.log"; exit 1; }
tail -1 "$O/utests.log"
bash tools/prof_rq.sh > /dev/null && python3 tools/trace_shapes.py "$O/prof/rqonly_kernel_trace.csv" unique_; python3 tools/trace_shapes.py "$O/prof/rqonly_kernel_trace.csv" rocclr && python3 -c "import json; print(json.load(open('$O/prof_rqonly.json'))['ms_per_step'])"
