set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; O="$R/gpurun_out"; mkdir -p "$O/attnf"
timeout -k 10 300 python -u -m pytest "$R/tests/test_jagged_attention_gpu.py" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/attnf/tests.log" 2>&1 || { tail -30 "$O/attnf/tests.log"; exit 1; }
tail -1 "$O/attnf/tests.log"
timeout -k 10 180 python3 -u "$R/tools/attn_probe.py" > "$O/attnf/probe.jsonl" 2> "$O/attnf/probe.err" || { tail "$O/attnf/probe.err"; exit 1; }
cat "$O/attnf/probe.jsonl"
timeout -k 10 400 python -u "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('rqvae', d['ms_per_step'], 'amazon', d['decoder_amazon']['ms_per_step'], 'ml32m b8', d['decoder_ml32m']['per_gpu_batch_8']['ms_per_step'], 'b64', d['decoder_ml32m']['per_gpu_batch_64']['ms_per_step'], d['decoder_ml32m']['per_gpu_batch_64']['kernels']['attention'])"
