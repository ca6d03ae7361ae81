"""Per-kernel register / LDS / scratch metadata from a hipcc device .s file.

usage: python tools/kmeta.py <file.s> [substring ...]"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    pats = sys.argv[2:]
    meta = s[s.index("amdhsa.kernels:"):]
    for ent in re.split(r"\n  - ", meta)[1:]:
        name = re.search(r"\.name:\s+(\S+)", ent)
        if not name or not all(p in name.group(1) for p in pats):
            continue
        f = dict(re.findall(r"\.(vgpr_count|agpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|"
                            r"group_segment_fixed_size|private_segment_fixed_size):\s+(\d+)", ent))
        print(name.group(1)[:70], f)


if __name__ == "__main__":
    main()
