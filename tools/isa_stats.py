"""Instruction mix and register use of kernels in a hipcc device assembly file.

usage: python tools/isa_stats.py <file.s> <substring-of-kernel-symbol> [...]
(make one with: hipcc -O3 -std=c++20 --offload-arch=gfx950 -I include
 --cuda-device-only -S csrc/<file>.hip -o /tmp/x.s)
"""
import re
import sys
from collections import Counter


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    s = open(path).read()
    names = re.findall(r"^(_Z\S+):", s, flags=re.M)
    for name in names:
        if not all(p in name for p in pats):
            continue
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        body = [l.strip() for l in s[i:j].split("\n") if l.strip() and not l.strip().startswith(";")]
        c = Counter(l.split()[0] for l in body if not l.endswith(":") and not l.startswith("."))
        k = s.find(".name:           " + name)
        meta = dict(re.findall(r"\.(vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count):\s+(\d+)",
                               s[max(0, k - 2500):k + 100])) if k >= 0 else {}
        print(name)
        print("  total %d  %s" % (sum(c.values()), meta))
        print("  " + ", ".join("%s %d" % kv for kv in c.most_common(14)))


if __name__ == "__main__":
    main()
