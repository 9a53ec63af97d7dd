#!/usr/bin/env python3
"""Derived per-kernel metrics from tools/pmc_summary.py output: VALU issue
utilisation (wave64 VALU = 2 cycles on a SIMD32), wait fractions, HBM bytes
(FETCH_SIZE x 2 on gfx950 + WRITE_SIZE, KB units)."""
import sys


def main():
    data, cur = {}, None
    for line in open(sys.argv[1]):
        if line.strip() and not line.startswith(" "):
            cur = line.strip()
            data[cur] = {}
        elif cur and line.strip():
            p = line.split()
            data[cur][p[0]] = float(p[1])
    for k, v in data.items():
        if "SQ_WAVE_CYCLES" not in v or "SQ_WAIT_ANY" not in v:
            continue
        wc = v["SQ_WAVE_CYCLES"]
        cyc = v.get("GRBM_GUI_ACTIVE", 0) / 8
        busy = v["SQ_INSTS_VALU"] / (1024 * cyc / 2) if cyc else 0
        print(f"{k[:58]:58s} cyc={cyc / 1e3:8.1f}K valu_busy={busy:4.2f} valu/wave={v['SQ_INSTS_VALU'] / v['SQ_WAVES']:7.0f} "
              f"lds/wave={v['SQ_INSTS_LDS'] / v['SQ_WAVES']:5.0f} salu/wave={v['SQ_INSTS_SALU'] / v['SQ_WAVES']:5.0f} "
              f"wait_any={v['SQ_WAIT_ANY'] / wc:4.2f} wait_inst={v['SQ_WAIT_INST_ANY'] / wc:4.2f} "
              f"active={v['SQ_ACTIVE_INST_ANY'] / wc:4.2f} hbm={(v.get('FETCH_SIZE', 0) * 2 + v.get('WRITE_SIZE', 0)) / 1e3:7.2f}MB"
              + (f" icache_miss={v['SQC_ICACHE_MISSES'] / max(v.get('SQC_ICACHE_REQ', 1), 1):5.3f}"
                 f" icache_req/wave={v.get('SQC_ICACHE_REQ', 0) / v['SQ_WAVES']:7.0f}" if "SQC_ICACHE_MISSES" in v else ""))


if __name__ == "__main__":
    main()
