"""Counter table of the persistent config-4 kernel across builds (rocprofv3 --pmc CSVs).

    python scripts/pmc_table.py gpurun_out/r6f2 > profiles/r6/pass_f/pmc_table.md

Expects <dir>/pmc_<build>_<group>/**/*counter_collection.csv and <dir>/pmc_<build>_<group>.json
(bench/pmc_persist.py's line: rows scored in the profiled dispatch).  For each build it sums
every counter over the persistent kernel's dispatch (the kernel whose name starts with
``persist``), normalises per 512-row item (rows / 512), and derives the ratios that locate
the bound: VALU / LDS / VMEM issue shares of the wave cycles, wait share, LDS bank conflicts
per LDS instruction, TA busy share of GPU-active cycles, mean L2 read latency, mean VMEM and
LDS instruction latency (level / count).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(dict)        # build -> counter -> value
    rows = {}
    kern = {}
    for sub in sorted(glob.glob(os.path.join(d, "pmc_*_*"))):
        if not os.path.isdir(sub):
            continue
        m = re.match(r"pmc_(.+)_(\d+)$", os.path.basename(sub))
        if not m:
            continue
        build = m.group(1)
        js = sub + ".json"
        try:
            line = [ln for ln in open(js) if ln.startswith("{")][-1]
            rows.setdefault(build, json.loads(line)["rows"])
        except (OSError, IndexError, KeyError, ValueError):
            pass
        for f in glob.glob(os.path.join(sub, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                short = re.sub(r"^void ", "", name).split("(")[0]
                if "persist" not in short:
                    continue
                kern[build] = short
                c = r["Counter_Name"]
                vals[build][c] = vals[build].get(c, 0.0) + float(r["Counter_Value"])
    return vals, rows, kern


def ratio(v, a, b):
    return v[a] / v[b] if a in v and b in v and v[b] else None


def main():
    d = sys.argv[1]
    vals, rows, kern = load(d)
    builds = [b for b in ("default", "readonly", "loader") if b in vals] + \
             [b for b in vals if b not in ("default", "readonly", "loader")]
    counters = sorted({c for b in builds for c in vals[b]})
    print("| counter | " + " | ".join(f"{b} (per 512-row item)" for b in builds) + " |")
    print("|---|" + "---|" * len(builds))
    for c in counters:
        cells = []
        for b in builds:
            v = vals[b].get(c)
            items = rows.get(b, 0) / 512
            cells.append("" if v is None else (f"{v / items:,.1f}" if items else f"{v:,.0f}"))
        print(f"| {c} | " + " | ".join(cells) + " |")
    derived = [
        ("VALU issue / wave cycles", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"),
        ("LDS issue / wave cycles", "SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES"),
        ("any issue / wave cycles", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"),
        ("waiting / wave cycles", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
        ("LDS bank conflicts / LDS instr", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS"),
        ("TA busy / GPU-active cycles (sum over TAs)", "TA_TA_BUSY_sum", "GRBM_GUI_ACTIVE"),
        ("TA stalled by TC / TA busy", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_TA_BUSY_sum"),
        ("L2 read latency (cycles / request)", "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum"),
        ("VMEM instr latency (level / instr)", "SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM"),
        ("LDS instr latency (level / instr)", "SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS"),
        ("VALU instr / row", "SQ_INSTS_VALU", None),
    ]
    print()
    print("| derived | " + " | ".join(builds) + " |")
    print("|---|" + "---|" * len(builds))
    for label, a, b in derived:
        cells = []
        for bd in builds:
            v = vals[bd]
            if b is None:
                x = v[a] / rows[bd] if a in v and rows.get(bd) else None
            else:
                x = ratio(v, a, b)
            cells.append("" if x is None else f"{x:.3f}")
        print(f"| {label} | " + " | ".join(cells) + " |")
    print()
    for b in builds:
        print(f"- {b}: `{kern.get(b, '?')}`, {rows.get(b, 0):,} rows in the profiled dispatch")


if __name__ == "__main__":
    main()
