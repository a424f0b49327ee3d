"""Instruction histogram of the outermost loops of a kernel's assembly (hipcc -S): blocks whose
LLVM annotation puts them in a 'Depth=1' loop (or one of its child loops).
Usage: python scripts/asm_hist.py <file.s> [top-N]"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
loops = {}                                   # depth-1 header -> set of member headers
cur_top = None
block_hdr = []                               # per line: the loop header of the block it is in
hdr = None
for i, l in enumerate(lines):
    m = re.match(r"(\.LBB\d+_\d+):\s+; =>This (?:Inner )?Loop Header: Depth=(\d+)", l)
    if m:
        name = m.group(1)[2:]
        hdr = name
        if m.group(2) == "1":
            cur_top = name
            loops[name] = {name}
            j = i + 1
            while j < len(lines) and re.match(r"\s+;\s+Child Loop", lines[j]):
                loops[name].add(re.search(r"Child Loop (BB\d+_\d+)", lines[j]).group(1))
                j += 1
    elif re.match(r"(\.LBB\d+_\d+:|; %bb\.\d+:)", l):
        mm = re.search(r"Header=(BB\d+_\d+) Depth=\d+", l)
        hdr = mm.group(1) if mm else None
    block_hdr.append(hdr)
for name, members in loops.items():
    body = [l.split()[0] for l, h in zip(lines, block_hdr)
            if h in members and l.startswith("\t") and not l.strip().startswith((".", ";"))]
    n = collections.Counter(body)
    cls = collections.Counter()
    for k, v in n.items():
        cls["s_nop" if k == "s_nop" else k.split("_")[0] + "_"] += v
    print(f"loop {name}: {len(body)} instructions; " + ", ".join(f"{k}{v}" for k, v in cls.most_common()))
    print("   exec/branch: " + ", ".join(f"{k} {n[k]}" for k in ("s_and_saveexec_b64", "s_or_b64", "s_andn2_b64",
                                                               "s_cbranch_execz", "s_cbranch_scc0", "s_cbranch_scc1",
                                                               "s_cbranch_vccz", "s_cbranch_vccnz", "s_branch")))
    print("   top: " + ", ".join(f"{k} {v}" for k, v in n.most_common(top)))
