"""VGPRs / SGPRs / scratch / occupancy per kernel of one HIP source, from the compiler's
kernel-resource-usage remarks.  Usage: kernel_resources.py file.hip [name-substring ...]
(KR_EXTRA: extra compiler flags, e.g. -D defines of an A/B build)"""
import re
import subprocess
import sys

src = sys.argv[1]
pats = sys.argv[2:]
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", *(["-fno-slp-vectorize"] if "raster" in src else []),
                    *[a for a in __import__("os").environ.get("KR_EXTRA", "").split() if a],
                    "-c", src, "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
                "LDS Size [bytes/block]"):
        m = re.search(re.escape(key) + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0]] = int(m.group(1))
for row in rows:
    n = subprocess.run(["c++filt", row["name"]], capture_output=True,
                       text=True).stdout.strip()
    n = re.sub(r"\((?!2\)).*$", "", n.replace("gs::(anonymous namespace)::", "").replace("float __vector(2)", "f2"))
    if pats and not any(p in n for p in pats):
        continue
    print(f"{n[:70]:70s} vgpr {row.get('VGPRs')} agpr {row.get('AGPRs')} sgpr {row.get('SGPRs')} "
          f"scratch {row.get('ScratchSize')} occ {row.get('Occupancy')} lds {row.get('LDS')}")
