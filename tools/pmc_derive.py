"""Derived per-kernel figures from tools/pmc_summary.py output (one file per
workload): instructions per wave by class, clock, VALU busy, L2 hit rate.
VALU busy = SQ_INSTS_VALU x 4 cycles / 1024 SIMDs / (clock x duration);
clock = GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md).

usage: python tools/pmc_derive.py gpurun_out/r6pmc/<workload>.txt [...] [--min-us 50]
"""
import re
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    min_us = 50.0
    if "--min-us" in sys.argv:
        min_us = float(sys.argv[sys.argv.index("--min-us") + 1])
        args = [a for a in args if a != sys.argv[sys.argv.index("--min-us") + 1]]
    for f in args:
        t = open(f).read()
        for blk in t.split("== ")[1:]:
            head = blk.split("\n")[0]
            v = {k: float(x) for k, x in re.findall(r"^\s+(\w+)\s+(\S+)$", blk, re.M)}
            if "_dur_ns" not in v or v["_dur_ns"] < min_us * 1e3 or not v.get("SQ_WAVES"):
                continue
            dur = v["_dur_ns"] * 1e-9
            clk = v["GRBM_GUI_ACTIVE"] / 8 / dur
            busy = v["SQ_INSTS_VALU"] * 4 / 1024 / (clk * dur)
            w = v["SQ_WAVES"]
            hit = v.get("TCC_HIT_sum", 0) / max(1.0, v.get("TCC_HIT_sum", 0) + v.get("TCC_MISS_sum", 0))
            name = head.split(" ", 1)[1] if " " in head else head
            print("%-58s %8.1f us  waves %8.0f  VALU/w %7.0f  SALU/w %6.0f  LDS/w %6.0f  VMEM/w %5.0f  "
                  "clk %.2f  VALU busy %.2f  L2 hit %.2f" % (
                      name[:58], dur * 1e6, w, v["SQ_INSTS_VALU"] / w, v["SQ_INSTS_SALU"] / w,
                      v.get("SQ_INSTS_LDS", 0) / w, v["SQ_INSTS_VMEM_RD"] / w, clk / 1e9, busy, hit))


if __name__ == "__main__":
    main()
