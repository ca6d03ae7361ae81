"""Per-chunk output bounds and agreed decision prefixes for the filter trace
fixtures (tests/golden/trace_*.npz).

filterL2's output is chaotic in the rounding: with every discrete decision
identical (the trace), the 50 multiplicative reweightings c *= 1 - tau/tau_max
(robust_estimator.py:167) carry a 1e-16 perturbation of the covariance to
1e-6 .. 1e-2 of max|out| at the end; and where a late iteration's top two
eigenvalues nearly coincide, even the removal decision becomes a function of
the rounding.  Both are measured per chunk with three independent fp64
evaluations of the reference's algorithm by the oracle (oracle/robust_np.py),
none of which is the reference's own sequential outer-product sum (:158):
the k x k covariance GEMM in two client orders ("gemm", "reverse") and the
n x n client-space form ("dual"):

  agree[chunk] = the number of leading iterations on which all three, and the
                 client-space form under four 1e-13 relative nudges of the
                 weights (oracle.trace_pair: a decision such a nudge flips is
                 a near-tie that rounding decides), make the reference's
                 decision (= the iteration count when they agree throughout);
  bound[chunk] = 3 * max over the three of |oracle - ref| / max|ref|.

The engine must reproduce the reference's decisions on the agreed prefix and
land within the bound (tests/test_gpu_filter_trace.py).  For ex_noregret
(not chaotic: the oracle lands 1e-13 .. 1e-12 from the reference) the bound
is 2e-5: the engine forms the step 0.5 / max|x_i - x_j|^2 (:54-58) from fp64
Gram distances rounded to fp32 while the reference rounds an fp32 BLAS norm,
and one fp32 ulp of the step moves the output by up to ~1e-5 of max.
Needs only numpy + the oracle.  Usage: python tests/golden/add_trace_bounds.py
"""
import glob
import json
import os
import sys
import warnings

# one BLAS thread: a threaded LAPACK/BLAS reduction order differs run to run,
# and these chaotic iterations turn that into different bounds
for _v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ[_v] = "1"

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import robust_np as orc  # noqa: E402


def main():
    for path in sorted(glob.glob(os.path.join(HERE, "trace_*.npz"))):
        z = dict(np.load(path))
        p = json.loads(str(z["params"]))
        func, x, ref = str(z["func"]), z["x"], z["out"]
        mode = 1 if func == "ex_noregret" else 0
        args = (list(x), p["eps"], p["sigma"], p["expansion"], p["itv"])
        outs, traces = [], []
        n = z["trace"].shape[1] // 2
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for order in (("gemm", "dual") if mode else ("gemm", "reverse", "dual")):
                tr = []
                if func == "ex_noregret":
                    outs.append(orc.ex_noregret(*args, trace=tr, order=order))
                elif func == "mom_filterL2":
                    outs.append(orc.mom_filterL2(*args, p["delta"], order=order, trace=tr))
                else:
                    outs.append(orc.filterL2(*args, order=order, trace=tr))
                traces.append(orc.trace_array(tr, mode, n))
            # rounding-sized nudges of the weights (oracle.trace_pair): a
            # decision they flip is a near-tie, outside the agreed prefix
            rows = x.reshape(x.shape[0], -1)
            if func == "mom_filterL2":
                num, size = orc.bucket_count(rows.shape[0], p["eps"], p["delta"])
                rows = np.asarray(orc.bucket_means(list(rows), size, num))
            extra = []
            for lo in range(0, rows.shape[1], p["itv"]):
                a, _, _ = orc.trace_pair((rows[:, lo:lo + p["itv"]], mode, p["eps"], p["sigma"], p["expansion"]))
                extra.append(a[:1 + n])
            traces.append(np.array(extra))
            for seed in range(orc.PERTURB_TRIALS):
                tr = []
                for lo in range(0, rows.shape[1], p["itv"]):
                    ch = rows[:, lo:lo + p["itv"]]
                    pt = (seed, orc.PERTURB_SCALE)
                    if mode:
                        orc.ex_noregret_(ch, p["eps"], p["sigma"], p["expansion"], trace=tr, order="dual", perturb=pt)
                    else:
                        orc.filterL2_(ch, p["eps"], p["sigma"], p["expansion"], order="dual", trace=tr, perturb=pt)
                traces.append(orc.trace_array(tr, mode, n))
        bound, agree = [], []
        for i, lo in enumerate(range(0, ref.shape[0], p["itv"])):
            sl = slice(lo, lo + p["itv"])
            m = np.abs(ref[sl]).max()
            far = max(np.abs(o[sl] - ref[sl]).max() for o in outs) / m
            bound.append(2e-5 if mode else 3.0 * far)
            want = z["trace"][i]
            a = int(want[0])
            for t in traces:
                diff = np.nonzero(t[i, 1:1 + want[0]] != want[1:1 + want[0]])[0]
                if t[i, 0] != want[0] or diff.size:
                    a = min(a, int(diff[0]) if diff.size else min(int(t[i, 0]), int(want[0])))
            agree.append(a)
        z["bound"] = np.array(bound)
        z["agree"] = np.array(agree, dtype=np.int32)
        np.savez_compressed(path, **z)
        print(os.path.basename(path), "bound", ["%.2e" % b for b in bound], "agree", agree,
              "iters", z["trace"][:, 0].tolist())


if __name__ == "__main__":
    main()
