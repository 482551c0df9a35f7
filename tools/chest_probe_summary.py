"""One-line-per-kernel summary of tools/chest_probe.py output files: python tools/chest_probe_summary.py <json>..."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f)
    for mode in d:
        for k in ("pilot", "stats"):
            x = d[mode][k]
            print("  %-8s %-6s span %6.1f us, wg median %6.1f |" % (mode, k, x["launch_span_us"], x["wg_us_median"]),
                  " ".join("%s %.1f" % (p, v["median_us"]) for p, v in x["phases"].items()))
        print("  %-8s reps pilot %s stats %s" % (mode, d[mode]["pilot_span_us_reps"], d[mode]["stats_span_us_reps"]))
