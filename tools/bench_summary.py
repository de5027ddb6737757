"""One summary row per bench.py JSON line found in the given log files."""
import json
import sys


def main(paths):
    for p in paths:
        try:
            lines = [l for l in open(p) if l.startswith("{")]
        except OSError:
            print(p, "missing")
            continue
        if not lines:
            print(p, "no JSON line")
            continue
        d = json.loads(lines[-1])
        c, r = d["config"], d.get("roofline") or {}
        print(p, c["workload"][:44], d["value"], d["ms_per_step"], "loops", c.get("loops"), r.get("kernel"),
              r.get("bound"), r.get("frac"), "traffic", r.get("traffic"),
              "fast", (d.get("fast_mode") or {}).get("value"), "cpu", (d.get("cpu_baseline") or {}).get("value"),
              "near", c.get("near_threshold_profiles"), "flips", c.get("mask_flips_vs_exact"),
              "exch", c.get("exchange_ms_per_step"))


if __name__ == "__main__":
    main(sys.argv[1:])
