"""One line per bench JSON (A/B runs): value, launch time, iterations per launch, kernel."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:   # noqa: BLE001
        print(f, "unreadable", e)
        continue
    r = d["roofline"]
    lc = d["config"]["launch"]
    print("%-28s %.3e  %8.1f us/launch  %6.2f us/it  frac %.3f  W%d zin%s  %s" % (
        f.split("/")[-1], d["value"], r["avg_launch_us"],
        r["avg_launch_us"] / r["iterations_per_launch"], r["frac"] or 0,
        lc["waves_per_group"], lc.get("zin"), lc["kernel"]))
