"""Summary of a bench.py JSON line (the last line starting with '{' of a file)."""
import json
import sys

d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
r = d["roofline"]
print(f"rqvae {d['ms_per_step']} ms  {d['value'] / 1e6:.2f} M items/s  gemm-roofline {r['shape']} {r['launch_ms']} ms "
      f"frac {r['frac']}  all-gemm {r['all_gemm_launches']}")
q = d.get("roofline_quantize", {})
print(f"quantize frac {q.get('frac')}  highest {d.get('exact_fp32_highest')}")
da = d.get("decoder_amazon", {})
if da:
    print(f"decoder_amazon {da['ms_per_step']} ms {da['ctx_tokens_per_s'] / 1e6:.3f} M ctx tok/s frac {da['roofline']['frac']} "
          f"attn {da['kernels']['attention']}")
dm = d.get("decoder_ml32m", {})
for k, v in dm.items():
    print(f"decoder_ml32m {k} {v['ms_per_step']} ms {v['ctx_tokens_per_s'] / 1e6:.3f} M ctx tok/s frac {v['roofline']['frac']}")
