#!/usr/bin/env python3
"""Derived per-dispatch PMC metrics from pmc_table.py output (csv on stdin)."""
import csv
import sys

for r in csv.DictReader(sys.stdin):
    f = {k: float(v) for k, v in r.items() if k not in ("kernel", "grid")}
    gui = f.get("GRBM_GUI_ACTIVE", 0) / 8
    wc = f.get("SQ_WAVE_CYCLES", 1) or 1
    out = f"{r['kernel'][:30]:30s} grid={r['grid']:>8s} cyc={gui:8.0f}"
    if gui:
        out += f" waves/CU={wc * 4 / gui / 256:5.1f}"
        out += f" TA={f.get('TA_TA_BUSY', 0) / 256 / gui:4.2f} TD={f.get('TD_TD_BUSY', 0) / 256 / gui:4.2f}"
    out += (f" wait={f.get('SQ_WAIT_ANY', 0) / wc:4.2f} waitI={f.get('SQ_WAIT_INST_ANY', 0) / wc:4.2f}"
            f" act={f.get('SQ_ACTIVE_INST_ANY', 0) / wc:4.2f}")
    if "TCP_TCC_READ_REQ" in f:
        out += f" rdlat={f['TCP_TCC_READ_REQ_LATENCY'] / max(f['TCP_TCC_READ_REQ'], 1):5.0f}"
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_LDS_BANK_CONFLICT"):
        if k in f:
            out += f" {k.replace('SQ_INSTS_', '').lower()}={f[k]:.3g}"
    print(out)
