#!/usr/bin/env python
"""One-line summary of a bench.py JSON output file (value, ms/step, schedule, memory)."""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(path, "unreadable:", e)
        continue
    c = d.get("config", {})
    keys = ("schedule", "schedule_probe_ms", "peak_mem_gb", "alloc_retries", "device_mallocs", "phase_ms")
    print(path, d.get("value"), d.get("unit"), d.get("ms_per_step"), {k: c.get(k) for k in keys})
