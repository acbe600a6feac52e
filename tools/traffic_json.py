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
    "mc": (["mc_kernel"], 8, 2),                      # 4-sample (8-B) window quads, per-pixel stores
    "itx": (["itx_frame_kernel"], 8, 8),              # 4-pixel chunks in and out
    "deblock": (["lf_tile_kernel"], 16, 16),           # uint4 tile staging and stores
    "cdef": (["cdef_kernel"], 16, 4),                 # 8-sample vectors in, pixel pairs out
    "lr": (["lr_kernel"], 16, 16),                    # 8-pixel vectors in and out
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
            t = k[3:-1].strip()
            width = {"unsigned short": 2, "unsigned int": 4, "HIP_vector_type<unsigned int, 2u>": 8,
                     "HIP_vector_type<unsigned int, 4u>": 16, "uint2": 8, "uint4": 16}.get(t)
            if width is None:
                continue
            if (kind == "rd") == (c == "FETCH_SIZE"):
                f[(c, width)] = CALIB_BYTES / (d[c] * 1024.0)
    return f


def sized_bytes(d):
    """Read bytes from the request-size counters: 32/64/128-B requests at their own size."""
    if "TCC_EA0_RDREQ_128B" not in d:
        return None
    return 32 * d.get("TCC_EA0_RDREQ_32B", 0.0) + 64 * d.get("TCC_EA0_RDREQ_64B", 0.0) + 128 * d["TCC_EA0_RDREQ_128B"]


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "pmc"     # the PMC passes' subdirectory
    fac = calib(root)
    fetch = collect(os.path.join(root, sub, "p1"))
    write = collect(os.path.join(root, sub, "p2"))
    req = collect(os.path.join(root, sub, "p3"))
    creq = collect(os.path.join(root, "calib_TCC_EA0_RDREQ"))
    # calibration of the sized count: true bytes / sized bytes per read width (expect 1.0)
    sized_cal = {}
    for k, d in creq.items():
        if k.startswith("rd<") and sized_bytes(d):
            sized_cal[k[3:-1].strip()] = round(CALIB_BYTES / sized_bytes(d), 4)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over "
                     "`bench.py --steps 5 --warmup 2` (pipeline only); counters in KB",
           "calibration": {f"{c}@{w}B": round(v, 4) for (c, w), v in sorted(fac.items())},
           "sized_read_calibration": sized_cal,
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
        ent = {"kernels": ks, "read_width": rw, "write_width": ww,
               "fetch_bytes_raw": int(fr), "write_bytes_raw": int(wr),
               "fetch_factor": round(fr_f, 4), "write_factor": round(wr_f, 4),
               "hbm_bytes_per_step_width_factor": int(fr * fr_f + wr * wr_f)}
        rd = None
        if all(k in req and sized_bytes(req[k]) is not None for k in ks):
            rd = sum(sized_bytes(req[k]) * req[k]["_dispatches"] for k in ks) / frames
            ent["read_bytes_sized"] = int(rd)
            ent["read_requests"] = {c: int(sum(req[k].get(c, 0.0) * req[k]["_dispatches"] for k in ks) / frames)
                                    for c in ("TCC_EA0_RDREQ", "TCC_EA0_RDREQ_32B", "TCC_EA0_RDREQ_64B",
                                              "TCC_EA0_RDREQ_128B")}
        # preferred: reads at their request sizes (calibrated to 1.0 on the streaming kernels), writes exact
        ent["hbm_bytes_per_step"] = int(rd + wr * wr_f) if rd is not None else ent["hbm_bytes_per_step_width_factor"]
        out["stages"][st] = ent
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
