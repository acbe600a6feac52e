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

    # inter prediction: a small 4:2:0 frame of MC units (single + compound) vs the oracle
    from rav1d_amd.frame import McMeta, mc_frame
    from rav1d_amd.synth import make_mc_units, make_texture
    rng = np.random.default_rng(7)
    w, h = 128, 96
    refs = []
    for _ in range(2):
        r = Frame(w, h, 10, 1)
        for p in range(3):
            pw, ph = r.dims(p)
            r.set_plane_np(p, make_texture(rng, pw, ph, 10))
        refs.append(r)
    units, cs, masks = make_mc_units(w, h, 1, rng, compound_frac=0.5, mv_px=16)
    cur = Frame(w, h, 10, 1)
    meta = McMeta(units, cs, masks)
    mc_frame(ctx, cur, refs, meta)
    torch.cuda.synchronize()
    exp, _ = oracle_lib.mc_frame([cur.buffer_np(p) * 0 for p in range(3)],
                                 [[r.buffer_np(p) for p in range(3)] for r in refs], 10, 1, w, h, units, masks)
    for p in range(3):
        if not np.array_equal(cur.buffer_np(p), exp[p]):
            raise AssertionError(f"smoke: mc plane {p} differs from the oracle")
