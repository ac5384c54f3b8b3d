"""Per-replayed-step kernel time by category from a rocprofv3 kernel trace: the launches between consecutive AdamW
kernels (one optimizer step each) of the last replays, so eager warm-up / capture steps do not count.

    python tools/step_breakdown.py gpurun_out/<tag>/prof/run_kernel_trace.csv [steps]
"""
import csv
import sys


def category(n):
    if "ppw_gemm" in n or "splitk_reduce" in n or "gemm_kernel<false, false" in n:
        return "wgrad GEMMs + reduce"
    if "gemm" in n:
        return "fwd/dgrad GEMMs"
    if "attn" in n:
        return "attention"
    if "ln_" in n or "slab_reduce" in n or "colsum" in n:
        return "LN + colsum"
    if "conv0" in n:
        return "conv0"
    if "adamw" in n or "sumsq" in n:
        return "adamw+clip"
    if "at::native" in n or "rocclr" in n:
        return "ATen/copies"
    return "other"


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    idx = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
    pairs = list(zip(idx[:-1], idx[1:]))[-(k + 1):-1] or list(zip(idx[:-1], idx[1:]))
    agg = {}
    for a, b in pairs:
        seg = rows[a + 1:b + 1]
        wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
        print(f"step: {len(seg)} kernels, wall {wall:.2f} ms")
        for r in seg:
            c = category(r["Kernel_Name"])
            agg[c] = agg.get(c, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    n = len(pairs)
    for c, v in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"  {c:24s} {v / n:6.2f} ms")
    print(f"  {'kernel sum':24s} {sum(agg.values()) / n:6.2f} ms")


if __name__ == "__main__":
    main()
