"""One line per bench JSON under gpurun_out/configs_<tag>/ (value, ms/step, CPU baseline)."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/configs_{sys.argv[1]}/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, round(d["value"] / 1e6, 2), "M", d["ms_per_step"], (d.get("cpu_baseline") or {}).get("value"))
    except Exception as e:  # noqa: BLE001
        print(f, "n/a", e)
