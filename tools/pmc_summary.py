"""Summarise rocprofv3 --pmc CSVs: per kernel, average counter value per dispatch."""
import csv, glob, os, sys, collections

def summarize(d, kernel_filter=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if kernel_filter and kernel_filter not in k:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_kernel_trace.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if kernel_filter and kernel_filter not in k:
                continue
            durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        if durs.get(k):
            out[k]["_dur_ns"] = sorted(durs[k])[len(durs[k]) // 2]
    return out

if __name__ == "__main__":
    for d in sys.argv[1:]:
        res = summarize(d, "sra::")
        for k, cs in res.items():
            print("==", d, k[:80])
            for c in sorted(cs):
                print("   %-26s %.4g" % (c, cs[c]))
