"""Summary of tools/orbit_policy.py output (JSON lines): how close the launch policy's own choice
('auto') comes to the fastest forced variant on every view, as one JSON object.
    python tools/orbit_policy_report.py run.jsonl [more.jsonl ...]"""
import json
import statistics
import sys


def report(path):
    rows = [json.loads(line) for line in open(path)]
    variants = [k for k, v in rows[0].items()
                if isinstance(v, float) and k not in ("yaw", "pitch", "radius")]
    auto = [r["auto"] for r in rows]
    best = [min(r[v] for v in variants) for r in rows]
    over = [a / b for a, b in zip(auto, best)]
    out = dict(file=path, views=len(rows), variants=variants,
               auto_sum_ms=round(sum(auto), 3), best_sum_ms=round(sum(best), 3),
               auto_over_best_sum=round(sum(auto) / sum(best), 4),
               auto_p50_ms=round(statistics.median(auto), 4), auto_max_ms=round(max(auto), 4),
               best_p50_ms=round(statistics.median(best), 4), best_max_ms=round(max(best), 4),
               views_auto_within_5pct=sum(o <= 1.05 for o in over),
               views_auto_over_20pct=sum(o > 1.20 for o in over),
               worst_auto_over_best=round(max(over), 3))
    for v in variants:
        if v != "auto":
            out[v + "_sum_ms"] = round(sum(r[v] for r in rows), 3)
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(json.dumps(report(p)))
