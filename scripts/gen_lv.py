"""Regenerate the LV accessors (prisma_engine.hip) from the Layout struct (engine_layout.h)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lay = open(os.path.join(ROOT, "prisma_amd/csrc/engine_layout.h")).read()
body = lay[lay.index("struct Layout {"):]
body = body[:body.index("};")]
fields = []
for line in body.splitlines():
    line = line.split("//")[0].strip()
    m = re.match(r"(int32_t|uint32_t|int64_t|double|float)\s+(.+);", line)
    if m:
        fields += [(n.strip(), m.group(1)) for n in m.group(2).split(",")]
acc = []
for n, t in fields:
    o = f"offsetof(Layout, {n}) / 4"
    if t in ("int32_t", "uint32_t"):
        acc.append(f"    __device__ __forceinline__ {t} {n}() const {{ return ({t})u({o}); }}")
    elif t == "float":
        acc.append(f"    __device__ __forceinline__ float {n}() const {{ return __uint_as_float(u({o})); }}")
    elif t == "int64_t":
        acc.append(f"    __device__ __forceinline__ int64_t {n}() const {{ return mk64(u({o}), u({o} + 1)); }}")
    else:
        acc.append(f"    __device__ __forceinline__ double {n}() const {{ return __longlong_as_double(mk64(u({o}), u({o} + 1))); }}")
p = os.path.join(ROOT, "prisma_amd/csrc/prisma_engine.hip")
s = open(p).read()
a = s.index("    __device__ __forceinline__ uint32_t u(int i) const")
a = s.index("\n", a) + 1
b = s.index("};", a)
s = s[:a] + "\n".join(acc) + "\n" + s[b:]
open(p, "w").write(s)
print(len(fields), "accessors")
