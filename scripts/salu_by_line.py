"""Static instruction counts by source line (a -gline-tables-only assembly file): where the scalar
(and vector) instructions of one kernel come from.  Usage: python scripts/salu_by_line.py file.s kernel_symbol [n]"""
import collections
import re
import sys

txt = open(sys.argv[1]).read()
name = sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
files = {}
for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', txt, re.M):
    files[m.group(1)] = (m.group(3) or m.group(2)).split('/')[-1]
m = re.search(rf"^{re.escape(name)}:[^\n]*\n(.*?)^\s*s_endpgm", txt, re.S | re.M)
cur = None
sal, val = collections.Counter(), collections.Counter()
tot = 0
for ln in m.group(1).splitlines():
    mm = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', ln)
    if mm:
        cur = (files.get(mm.group(1), mm.group(1)), int(mm.group(2)))
        continue
    if ln.startswith('\t') and not ln.strip().startswith(('.', ';')):
        op = ln.strip().split()[0]
        tot += 1
        if op.startswith('s_') and not op.startswith(('s_waitcnt', 's_nop', 's_cbranch', 's_branch')):
            sal[cur] += 1
        elif op.startswith('v_'):
            val[cur] += 1
print('total', tot, 'salu', sum(sal.values()), 'valu', sum(val.values()))
for k, v in sal.most_common(n):
    print(v, val[k], k)
