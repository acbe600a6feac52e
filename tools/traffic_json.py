"""HBM bytes per bench step from tools/gpu_profile.sh's PMC passes, calibrated per access width.

usage: python tools/traffic_json.py <profile dir>   (prints JSON; commit it as profiles/r01_traffic.json)

<dir>/calib_FETCH_SIZE, calib_WRITE_SIZE: tools/pmc_calib (1 GiB streamed per kernel, widths
2/4/8/16 B per lane) -> factor(width) = true bytes / (counter KB * 1024), per MI355X_MICROARCH.md
"calibrate on a known byte count in your own access pattern".
<dir>/pmc/p1 (FETCH_SIZE), <dir>/pmc/p2 (WRITE_SIZE): the bench. Per kernel the mean counter per
dispatch; per stage per step = the stage's counter total / frames run, scaled by the
factor of the stage's dominant global access width (the widths the kernels' source uses).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import collect  # noqa: E402

CALIB_BYTES = 1 << 30
# stage -> (kernel name prefixes, dominant read width, dominant write width in bytes)
STAGES = {
    "mc": (["mc_kernel"], 2, 2),                      # per-pixel u16 window gathers
    "itx": (["itx_frame_kernel"], 8, 2),
    "deblock": (["lf_cols_kernel", "lf_rows_kernel"], 2, 2),
    "cdef": (["cdef_kernel"], 8, 8),                  # uint2 tile rows
    "lr": (["lr_kernel"], 2, 2),
}
FRAME_KERNEL = "cdef_kernel"                          # one dispatch per frame: counts the frames


def calib(root):
    f = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        res = collect(os.path.join(root, f"calib_{c}"))
        for k, d in res.items():
            kind = "rd" if k.startswith("rd<") else "wr" if k.startswith("wr<") else None
            if kind is None or c not in d:
                continue
            t = k[3:].rstrip(">")
            width = {"unsigned short": 2, "unsigned int": 4, "HIP_vector_type<unsigned int, 2u>": 8,
                     "HIP_vector_type<unsigned int, 4u>": 16, "uint2": 8, "uint4": 16}.get(t)
            if width is None:
                continue
            if (kind == "rd") == (c == "FETCH_SIZE"):
                f[(c, width)] = CALIB_BYTES / (d[c] * 1024.0)
    return f


def main():
    root = sys.argv[1]
    fac = calib(root)
    fetch = collect(os.path.join(root, "pmc", "p1"))
    write = collect(os.path.join(root, "pmc", "p2"))
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over "
                     "`bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fg`; counters in KB",
           "calibration": {f"{c}@{w}B": round(v, 4) for (c, w), v in sorted(fac.items())},
           "kernels": {}, "stages": {}}
    for k in sorted(set(fetch) | set(write)):
        out["kernels"][k] = {"dispatches": fetch.get(k, {}).get("_dispatches"),
                             "fetch_kb_per_dispatch": round(fetch.get(k, {}).get("FETCH_SIZE", 0.0), 1),
                             "write_kb_per_dispatch": round(write.get(k, {}).get("WRITE_SIZE", 0.0), 1)}
    frames = next((d["_dispatches"] for k, d in fetch.items() if k.startswith(FRAME_KERNEL)), None)
    out["frames"] = frames
    for st, (pre, rw, ww) in STAGES.items():
        ks = [k for k in fetch if any(k.startswith(p) for p in pre)]
        if not frames or not ks or not all(k in write for k in ks):
            continue
        fr = sum(fetch[k]["FETCH_SIZE"] * fetch[k]["_dispatches"] for k in ks) * 1024 / frames
        wr = sum(write[k]["WRITE_SIZE"] * write[k]["_dispatches"] for k in ks) * 1024 / frames
        fr_f, wr_f = fac.get(("FETCH_SIZE", rw), 1.0), fac.get(("WRITE_SIZE", ww), 1.0)
        out["stages"][st] = {"kernels": ks, "read_width": rw, "write_width": ww,
                             "fetch_bytes_raw": int(fr), "write_bytes_raw": int(wr),
                             "fetch_factor": round(fr_f, 4), "write_factor": round(wr_f, 4),
                             "hbm_bytes_per_step": int(fr * fr_f + wr * wr_f)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
