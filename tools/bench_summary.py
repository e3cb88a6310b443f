#!/usr/bin/env python3
"""One screen of a bench.py JSON line: the headline, the roofline, the alternative mode, the other
configs, multi-GPU, CPU baseline.    python3 tools/bench_summary.py bench.json"""
import json
import sys


def main():
    d = json.loads([l for l in open(sys.argv[1]) if l.strip().startswith("{")][-1])
    r = d.get("roofline") or {}
    print(f"{d['config'].get('name')} {d['config'].get('coeff_mode')} n_gpus={d['n_gpus']} value={d['value']:.4g} "
          f"ms={d['ms_per_step']} parity_ok={d.get('parity_ok')} roofline {r.get('kernel')} frac={r.get('frac')}")
    print("  phases", d.get("phase_ms_per_call"))
    for m, a in (d.get("alt_modes") or {}).items():
        rv = a.get("roofline_valu") or {}
        print(f"  alt {m}: ms={a['ms_per_step']} phases={a['phase_ms_per_call']} "
              f"call_issue={(rv.get('call_issue') or {}).get('frac')}")
    for n, o in (d.get("other_configs") or {}).items():
        rf = o.get("roofline") or o.get("roofline_valu") or {}
        print(f"  {n}: ms={o['ms_per_step']} parity_ok={o.get('parity_ok')} frac={rf.get('frac')} "
              f"traffic={rf.get('traffic')} call_frac={(rf.get('call') or {}).get('frac')}"
              + (f" cpu_ref={o['cpu_reference']}" if 'cpu_reference' in o else "")
              + (f" same_plane={o['same_plane_1gpu']['ms_per_step']}" if o.get('same_plane_1gpu') else "")
              + (f" long_run={ {k: o['long_run'][k] for k in ('steps', 'total_s', 'steady_ms_per_call')} }"
                 if o.get('long_run') else ""))
    m = d.get("multi_gpu")
    if m:
        print(f"  multi: rccl_ranks={m['rccl_ranks']} rank_ms={m['rank_ms_per_step']} halo={m['halo_ms_per_call']} "
              f"same_plane={d.get('ms_per_step_1gpu_same_plane')} speedup={d.get('speedup')}")
    c = d.get("cpu_baseline")
    if c:
        print(f"  cpu: {c.get('value')} {c.get('kind')} s/call={c.get('s_per_call')} sample={c.get('sample')} "
              f"col_sample={(c.get('column_sample') or {}).get('sample_over_whole')}")


if __name__ == "__main__":
    main()
