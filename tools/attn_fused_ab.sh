set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out/attnf"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest "$R/tests/test_jagged_attention_gpu.py" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
bash "$R/tools/attn_ab.sh" "$@"
