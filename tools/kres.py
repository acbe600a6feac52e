"""Print per-kernel resource usage (VGPRs, spills, occupancy, LDS) of one HIP source for gfx950.
    python tools/kres.py rav1d_amd/csrc/itx.hip [name-substring]"""
import re, subprocess, sys, os
src = os.path.abspath(sys.argv[1])
inc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "include")
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + inc, "-c", src,
                    "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("MI_EXTRA_FLAGS", "").split() + (["-xhip"] if src.endswith(".cpp") else []),
                   capture_output=True, text=True, cwd="/tmp")
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for c in rows:
    if flt in c["name"]:
        dem = subprocess.run(["c++filt", c["name"]], capture_output=True, text=True).stdout.strip()
        print(f"{dem[:90]:90s} vgpr={c.get('VGPRs')} agpr={c.get('AGPRs')} spill={c.get('VGPRs Spill')} "
              f"scratch={c.get('ScratchSize [bytes/lane]')} occ={c.get('Occupancy [waves/SIMD]')} lds={c.get('LDS Size [bytes/block]')}")
