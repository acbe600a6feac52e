"""One small pass of every implemented stage on cuda:0, checked bit-exactly against the
oracle. Used by __graft_entry__.smoke()."""


def run_smoke(ctx, oracle_lib, np, torch):
    from rav1d_amd.frame import Frame, itx_frame
    from rav1d_amd.synth import make_itx_frame

    fr = make_itx_frame(128, 96, bpc=10, seed=42)
    f = Frame(fr["w"], fr["h"], fr["bpc"], fr["layout"])
    for p, arr in enumerate(fr["planes"]):
        f.set_plane_np(p, arr)
    blocks = torch.from_numpy(fr["blocks"].view(np.uint8).copy()).cuda()
    coef = torch.from_numpy(fr["coef"].copy()).cuda()
    itx_frame(ctx, f, blocks, fr["size_start"], coef)
    torch.cuda.synchronize()
    ref = oracle_lib.itx_frame([p.copy() for p in fr["planes"]], fr["blocks"], fr["coef"].copy(), 10)
    for p in range(3):
        if not np.array_equal(f.plane_np(p), ref[p]):
            raise AssertionError(f"smoke: itx plane {p} differs from the oracle")
