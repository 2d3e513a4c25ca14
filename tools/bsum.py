"""One-line summary of bench.py JSON lines in the given logs: img/s, ms/step, GEMM frac, head+loss fwd frac."""
import json
import sys

for path in sys.argv[1:]:
    for ln in open(path):
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        rl = d.get("roofline_loss", {})
        hk = rl.get("head_loss_fwd_kernel_live", {})
        hc = rl.get("head_loss_fwd_live", {})
        lf = rl.get("pis_loss_fwd_cold", {})
        print(f"{path}: {d['value']:.1f} img/s {d['ms_per_step']:.3f} ms  gemm {d['roofline_gemm']['frac']:.3f} "
              f"({d['roofline_gemm']['ms_per_step']:.2f} ms)  hl_fwd kernel {hk.get('frac', 0):.3f} "
              f"({hk.get('avg_launch_ms', 0) * 1e3:.1f} us) call {hc.get('frac', 0):.3f} "
              f"({hc.get('avg_call_ms', 0) * 1e3:.1f} us)  loss_fwd/floor {lf.get('floor', {}).get('loss_over_floor', 0):.2f}"
              f"  mode {d.get('step_mode', 'eager')[:9]} eager {d.get('ms_per_step_eager') or 0:.3f} ms")
