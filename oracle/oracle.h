/*
 * oracle.h — CPU restatement of rav1d's DSP hot path. TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker for the HIP path in rav1d_amd/. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * library (rav1d_amd/librav1d_amd.so) never links or calls it.
 *
 * Each function restates the scalar reference implementation (the Rust `*_rust`/`*_c`
 * fallbacks in FreezyLemon/rav1d, identical to the same-commit dav1d C templates) and
 * cites the reference file:line it follows.
 *
 * Parity pinning status: see DESIGN.md §Oracle. The reference's C build needs the
 * meson-generated config.h, so per the project rules it is unbuildable here; the
 * restatement is pinned by the reference's own fixtures only where the repo's
 * front-end can replay them (not yet) — until then it is "parity unpinned".
 *
 * Conventions (as the reference): pixels are uint8_t (bpc 8) or uint16_t (bpc 10/12),
 * strides are in BYTES (BD::pxstride, include/common/bitdepth.rs:113-125), coefficients
 * are int16_t (bpc 8) or int32_t (bpc 10/12) (bitdepth.rs:272-401).
 */
#ifndef MI_ORACLE_H
#define MI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- itx (src/itx.rs, src/itx_1d.rs; C twin src/itx_tmpl.c, src/itx_1d.c) ---- */
/* One table entry: itxfm_add[tx][txtp](dst, stride, coeff, eob, bitdepth_max).  */
void oracle_itxfm_add(int tx, int txtp, void *dst, ptrdiff_t stride, void *coeff,
                      int eob, int bitdepth_max);
/* Frame-batched form used by the parity tests: blocks as in include/mi_av1dsp.h. */
void oracle_itx_frame(void *const planes[3], const ptrdiff_t strides[3],
                      const void *blocks, int n_blocks, void *coef_arena,
                      int bitdepth_max);
/* 1-D transforms exposed for the numeric sanity tests (kind: 0 dct,1 adst,2 flipadst,3 identity,4 wht) */
void oracle_itx_1d(int kind, int n, int32_t *c, ptrdiff_t stride, int min, int max);

#ifdef __cplusplus
}
#endif
#endif
