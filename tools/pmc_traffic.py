"""Collect a profiling session (tools/profile_round.sh) into profiles/.

For every workload: copies the rocprofv3 kernel stats CSV to
profiles/<tag>_<workload>_kernel_stats.csv; for the PMC workloads computes
the per-launch HBM bytes of the dominant kernel,
    traffic = 2 * FETCH_SIZE + WRITE_SIZE   (bytes; FETCH_SIZE is reported in
    KiB and counts half the bytes of wide coalesced reads on gfx950,
    MI355X_MICROARCH.md HBM/rocprofv3 section),
and merges it into profiles/traffic.json under "agg:N=<n>:d=<d>".

Usage: python tools/pmc_traffic.py gpurun_out/prof_r01 [tag]
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOMINANT = {"trimmedmean": "select_plain_kernel", "median": "select_plain_kernel", "average": "average",
            "trimmedmean_n100": "select_plain_kernel", "median_n100": "select_plain_kernel",
            "trimmedmean_n512": "select_quad_kernel", "median_n512": "select_quad_kernel",
            "krum": "gram_glds_kernel", "dba_median": "select_reg_kernel", "dba_weighted_sum": "rows_vec4_kernel"}
# Whole-op workloads (bench.py prices the whole call): traffic = the sum over
# every sra:: dispatch of a call, the calls counted by one anchor launch each
# (launches under 10 % of the largest anchor's fetch are bench.py's small
# side calls, e.g. the solver-flop probe on 1000 columns, and are not counted)
WHOLE_OP = {"filterl2": "chunk_gram", "ex_noregret": "chunk_gram", "mom_filterl2": "chunk_gram",
            "mom_ex_noregret": "chunk_gram", "bulyankrum": "gram_glds_kernel", "mom_krum": "gram_bucket_kernel",
            "bulyanmedian": "bulyan_final", "bulyantrimmedmean": "bulyan_final"}


def _find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return hits[0] if hits else None


def bench_line(logf):
    for ln in open(logf):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


def pmc_mean(d, kernel_sub):
    f = _find(d, "*counter_collection.csv")
    if not f:
        return None, None
    vals, name = [], None
    for r in csv.DictReader(open(f)):
        if kernel_sub in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
            name = r["Kernel_Name"]
    return (sum(vals) / len(vals) if vals else None), name


def whole_op(d, anchor):
    """(mean KiB per call over all sra:: dispatches, number of calls, per-kernel KiB/launch)."""
    f = _find(d, "*counter_collection.csv")
    if not f:
        return None, 0, {}
    rows = [r for r in csv.DictReader(open(f)) if "sra::" in r["Kernel_Name"]]
    anch = [float(r["Counter_Value"]) for r in rows if anchor in r["Kernel_Name"]]
    if not anch:
        return None, 0, {}
    calls = sum(1 for v in anch if v >= 0.1 * max(anch))
    per = {}
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        c = per.setdefault(k, [0.0, 0])
        c[0] += float(r["Counter_Value"])
        c[1] += 1
    tot = sum(float(r["Counter_Value"]) for r in rows)
    return tot / calls, calls, {k: (v[0] / calls, v[1]) for k, v in per.items()}


def main():
    src = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(src.rstrip("/"))
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    for logf in sorted(glob.glob(os.path.join(src, "*.log"))):
        name = os.path.basename(logf)[:-4]
        if name.startswith("pmc_"):
            continue
        st = _find(os.path.join(src, name), "*kernel_stats.csv")
        if st:
            shutil.copy(st, os.path.join(prof, "%s_%s_kernel_stats.csv" % (tag, name)))
        line = bench_line(logf)
        if line:
            with open(os.path.join(prof, "%s_%s_bench.json" % (tag, name)), "w") as fh:
                json.dump(line, fh, indent=1)
    tj_path = os.path.join(prof, "traffic.json")
    tj = json.load(open(tj_path)) if os.path.exists(tj_path) else {}
    for d in sorted(glob.glob(os.path.join(src, "pmc_*_FETCH_SIZE"))):
        name = re.match(r"pmc_(.*)_FETCH_SIZE", os.path.basename(d)).group(1)
        lp = os.path.join(src, "%s.log" % name)
        line = bench_line(lp) if os.path.exists(lp) else None
        if line is None:   # a PMC-only session: the bench line of the counter run itself
            line = bench_line(os.path.join(src, "pmc_%s_FETCH_SIZE.log" % name))
        if line is None:
            continue
        cfg = line["config"]
        key = "%s:N=%d:d=%d" % (cfg["aggregator"], cfg["clients"], cfg["d_per_gpu"])
        agg = cfg["aggregator"]
        if agg in WHOLE_OP:
            fetch_kib, calls, per_f = whole_op(d, WHOLE_OP[agg])
            write_kib, _, per_w = whole_op(os.path.join(src, "pmc_%s_WRITE_SIZE" % name), WHOLE_OP[agg])
            if fetch_kib is None or write_kib is None:
                continue
            traffic = 2 * fetch_kib * 1024 + write_kib * 1024
            sec = line["roofline"].get("secondary") or {}
            alg_b = line["roofline"].get("algorithmic_bytes_per_launch") or sec.get("algorithmic_bytes_per_launch")
            tj[key] = {"kernel": "whole op (all sra:: dispatches of one call; %d calls)" % calls,
                       "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
                       "hbm_bytes_per_launch": traffic, "algorithmic_bytes_per_launch": alg_b,
                       "per_kernel_bytes_per_call": {k: {"read": 2 * v[0] * 1024,
                                                         "write": per_w.get(k, (0.0, 0))[0] * 1024,
                                                         "launches": v[1]} for k, v in per_f.items()},
                       "note": "per call: 2*FETCH_SIZE + WRITE_SIZE summed over the call's kernels "
                               "(gfx950 FETCH_SIZE counts half of wide reads)",
                       "source": tag}
        else:
            sub = DOMINANT.get(name, "sra::")
            fetch_kib, kname = pmc_mean(d, sub)
            write_kib, _ = pmc_mean(os.path.join(src, "pmc_%s_WRITE_SIZE" % name), sub)
            if fetch_kib is None or write_kib is None:
                continue
            traffic = 2 * fetch_kib * 1024 + write_kib * 1024
            tj[key] = {"kernel": kname, "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
                       "hbm_bytes_per_launch": traffic,
                       "algorithmic_bytes_per_launch": line["roofline"].get("algorithmic_bytes_per_launch"),
                       "note": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of wide reads)",
                       "source": tag}
        print(key, "traffic %.4g B/launch" % traffic)
    with open(tj_path, "w") as fh:
        json.dump(tj, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
