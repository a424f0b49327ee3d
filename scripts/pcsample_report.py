"""Summarise a rocprofv3 PC-sampling CSV (scripts/pcsample.sh): samples per instruction class
and the hottest instructions of the step kernel.  A time-based host-trap sample lands on the
instruction a wave is about to issue, so a class's share of samples is its share of wave time
(issue and the stalls in front of it).

Usage: python scripts/pcsample_report.py <pc_sampling csv> [kernel-name substring] [top N]
"""
import collections
import csv
import sys


def classify(ins: str) -> str:
    op = ins.split()[0] if ins else "?"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_store")):
        return "smem"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "lane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else ""
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("no samples")
        return
    cols = list(rows[0].keys())
    print("columns:", cols)
    icol = next((c for c in cols if c.lower() in ("instruction", "inst")), None)
    ocol = next((c for c in cols if "offset" in c.lower() or c.lower() in ("pc", "pc_address")), None)
    kcol = next((c for c in cols if "kernel" in c.lower() and "name" in c.lower()), None)
    if kern and kcol:
        rows = [r for r in rows if kern in r[kcol]]
    n = len(rows)
    print(f"{n} samples" + (f" in kernels matching {kern!r}" if kern else ""))
    cls = collections.Counter(classify(r.get(icol, "")) for r in rows)
    for c, k in cls.most_common():
        print(f"  {c:8s} {k:8d}  {k / n:6.1%}")
    hot = collections.Counter((r.get(ocol, ""), r.get(icol, "")) for r in rows)
    print(f"top {top} instructions (offset, text, samples, share):")
    for (off, ins), k in hot.most_common(top):
        print(f"  {off:>10s}  {ins[:70]:70s} {k:7d} {k / n:6.2%}")


if __name__ == "__main__":
    main()
