"""Extract the normative AV1 entropy-decoding data (default CDFs, scan orders, dequantizer and
quantizer-matrix tables) from the reference's C twin into data includes for the host front-end
(rav1d_amd/host/tables/*.inc). Only numbers are emitted; the front-end's code is its own.
Run in the survey container (the reference does not exist on the GPU box); the generated
files are committed.

  python tools/gen_dec_tables.py [/root/reference/src]

Sources: src/cdf.c (av1_default_cdf, default_kf_y_mode_cdf, av1_default_coef_cdf[4],
default_mv_component_cdf, default_mv_joint_cdf; field shapes from src/cdf.h), src/scan.c,
src/dequant_tables.c, src/qm.c. The CDF tables are stored as the reference stores them:
32768 - cdf, with a zero adaptation counter in slot n_symbols.
"""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "rav1d_amd", "host", "tables")

CONST = dict(N_INTRA_PRED_MODES=13, N_UV_INTRA_PRED_MODES=14, N_BL_LEVELS=5, N_PARTITIONS=10,
             N_COMP_INTER_PRED_MODES=8, DAV1D_MAX_SEGMENTS=8, DAV1D_N_SWITCHABLE_FILTERS=3,
             N_TX_SIZES=5, N_BS_SIZES=22, N_MV_JOINTS=4, N_RECT_TX_SIZES=19, QINDEX_RANGE=256)
BS_NAMES = ["BS_128x128", "BS_128x64", "BS_64x128", "BS_64x64", "BS_64x32", "BS_64x16", "BS_32x64",
            "BS_32x32", "BS_32x16", "BS_32x8", "BS_16x64", "BS_16x32", "BS_16x16", "BS_16x8", "BS_16x4",
            "BS_8x32", "BS_8x16", "BS_8x8", "BS_8x4", "BS_4x16", "BS_4x8", "BS_4x4"]
ENUM = {n: i for i, n in enumerate(BS_NAMES)}


def strip_comments(t):
    t = re.sub(r"/\*.*?\*/", "", t, flags=re.S)
    return re.sub(r"//[^\n]*", "", t)


def body(txt, decl):
    """Initializer text (between the outer braces) of the definition whose text contains decl."""
    i = txt.index(decl)
    j = txt.index("=", i)
    k = txt.index("{", j)
    depth, m = 0, k
    while True:
        c = txt[m]
        depth += c == "{"
        depth -= c == "}"
        m += 1
        if depth == 0:
            return txt[k:m]


TOK = re.compile(r"\s*(?:(?P<num>-?\s*\d+)|(?P<id>[A-Za-z_]\w*)|(?P<p>[{}\[\](),=.]))")


def tokens(s):
    out, pos = [], 0
    while pos < len(s):
        m = TOK.match(s, pos)
        if not m:
            if s[pos:].strip() == "":
                break
            raise ValueError(s[pos:pos + 40])
        pos = m.end()
        if m.group("num") is not None:
            out.append(("n", int(m.group("num").replace(" ", ""))))
        elif m.group("id") is not None:
            out.append(("i", m.group("id")))
        else:
            out.append(("p", m.group("p")))
    return out


class P:
    """Parser of a C aggregate initializer into nested lists of (designator, value) items;
    CDFn(a, ...) expands to the stored form 32768 - a, ..."""

    def __init__(self, toks):
        self.t, self.k = toks, 0

    def peek(self):
        return self.t[self.k] if self.k < len(self.t) else (None, None)

    def eat(self, v=None):
        tok = self.t[self.k]
        if v is not None:
            assert tok[1] == v, (tok, v, self.t[self.k - 5:self.k + 5])
        self.k += 1
        return tok

    def value(self):
        kind, v = self.peek()
        if v == "{":
            return [self.items()]
        if kind == "i" and v.startswith("CDF"):
            self.eat()
            self.eat("(")
            vals = []
            while self.peek()[1] != ")":
                vals.append(32768 - self.eat()[1])
                if self.peek()[1] == ",":
                    self.eat(",")
            self.eat(")")
            return vals
        if kind == "i":
            self.eat()
            return [ENUM[v]]
        self.eat()
        return [v]

    def items(self):
        self.eat("{")
        out = []
        while self.peek()[1] != "}":
            desig = None
            if self.peek()[1] == "[":
                self.eat("[")
                kind, v = self.eat()
                desig = ("idx", ENUM[v] if kind == "i" else v)
                self.eat("]")
                self.eat("=")
            elif self.peek()[1] == ".":
                self.eat(".")
                desig = ("field", self.eat()[1])
                self.eat("=")
            for j, v in enumerate(self.value()):
                out.append((desig if j == 0 else None, v))
            if self.peek()[1] == ",":
                self.eat(",")
        self.eat("}")
        return out


def fill(arr, items):
    """C aggregate initialization of ndarray arr from parsed items (no brace elision except a
    run of scalars at the innermost level)."""
    pos = 0
    for desig, v in items:
        if desig is not None:
            pos = desig[1]
        if isinstance(v, list):
            fill(arr[pos], v)
        else:
            assert arr.ndim == 1, "brace elision above the innermost level"
            arr[pos] = v
        pos += 1


def fields_of(items):
    out = {}
    for desig, v in items:
        assert desig is not None and desig[0] == "field"
        out[desig[1]] = v
    return out


def struct_dims(hdr, name):
    m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), hdr, flags=re.S)
    dims = []
    for f, d in re.findall(r"ALIGN\(uint16_t (\w+)((?:\[[^\]]+\])+), \d+\)", m.group(1)):
        shape = [eval(x, {}, CONST) for x in re.findall(r"\[([^\]]+)\]", d)]
        dims.append((f, shape))
    return dims


def emit(lines, name, arr, ctype="uint16_t"):
    flat = [int(v) for v in np.asarray(arr).ravel()]
    lines.append(f"static const {ctype} {name}[{len(flat)}] = {{")
    for k in range(0, len(flat), 16):
        lines.append("    " + ", ".join(str(v) for v in flat[k:k + 16]) + ",")
    lines.append("};")


def gen_cdf(src, lines):
    txt = strip_comments(open(os.path.join(src, "cdf.c")).read())
    hdr = strip_comments(open(os.path.join(src, "cdf.h")).read())
    mode = fields_of(P(tokens(body(txt, "CdfModeContext av1_default_cdf"))).items())
    for f, shape in struct_dims(hdr, "CdfModeContext"):
        a = np.zeros(shape, np.int64)
        fill(a, mode[f])
        emit(lines, f"k_cdf_mode_{f}", a)
    kf = np.zeros((5, 5, 16), np.int64)
    fill(kf, P(tokens(body(txt, "default_kf_y_mode_cdf["))).items())
    emit(lines, "k_cdf_kf_y_mode", kf)
    coef_items = P(tokens(body(txt, "CdfCoefContext av1_default_coef_cdf[4]"))).items()
    coef_dims = struct_dims(hdr, "CdfCoefContext")
    for q, (desig, v) in enumerate(coef_items):
        assert desig == ("idx", q)
        fl = fields_of(v)
        for f, shape in coef_dims:
            a = np.zeros(shape, np.int64)
            fill(a, fl[f])
            emit(lines, f"k_cdf_coef{q}_{f}", a)
    mvc = fields_of(P(tokens(body(txt, "CdfMvComponent default_mv_component_cdf"))).items())
    for f, shape in struct_dims(hdr, "CdfMvComponent"):
        a = np.zeros(shape, np.int64)
        fill(a, mvc[f])
        emit(lines, f"k_cdf_mv_{f}", a)
    j = np.zeros(4, np.int64)
    fill(j, P(tokens(body(txt, "default_mv_joint_cdf["))).items())
    emit(lines, "k_cdf_mv_joint", j)


def gen_scan(src, lines):
    txt = strip_comments(open(os.path.join(src, "scan.c")).read())
    for w, h in [(4, 4), (8, 8), (16, 16), (32, 32), (4, 8), (8, 4), (8, 16), (16, 8), (16, 32), (32, 16),
                 (4, 16), (16, 4), (8, 32), (32, 8)]:
        n = w * h
        a = np.zeros(n, np.int64)
        fill(a, P(tokens(body(txt, f"scan_{w}x{h}[]"))).items())
        assert sorted(a.tolist()) == list(range(n))
        emit(lines, f"k_scan_{w}x{h}", a)


def gen_dq(src, lines):
    txt = strip_comments(open(os.path.join(src, "dequant_tables.c")).read())
    a = np.zeros((3, 256, 2), np.int64)
    fill(a, P(tokens(body(txt, "dav1d_dq_tbl["))).items())
    emit(lines, "k_dq_flat", a)


def gen_qm(src, lines):
    """dav1d_qm_tbl[15][2][tx] expanded as dav1d_init_qm_tables does (qm.c:3079-3148): stored
    transposed, 4x4 / 8x8 / 32x32 from lower triangles, 16x16 subsampled from 32x32."""
    txt = strip_comments(open(os.path.join(src, "qm.c")).read())

    def load(name, n):
        a = np.zeros((15, 2, n), np.int64)
        fill(a, P(tokens(body(txt, f"{name}[][2][{n}]"))).items())
        return a

    def untri(t, sz):
        out = np.zeros((sz, sz), np.int64)
        for y in range(sz):
            for x in range(sz):
                # symmetric matrix stored as the lower triangle, row by row
                a, b = (y, x) if x <= y else (x, y)
                out[y, x] = t[a * (a + 1) // 2 + b]
        return out.ravel()

    t44, t84, t88 = load("qm_tbl_4x4_t", 10), load("qm_tbl_8x4", 32), load("qm_tbl_8x8_t", 36)
    t164, t168, t328 = load("qm_tbl_16x4", 64), load("qm_tbl_16x8", 128), load("qm_tbl_32x8", 256)
    t3216, t3232 = load("qm_tbl_32x16", 512), load("qm_tbl_32x32_t", 528)
    # tx order: TX_4X4, 8X8, 16X16, 32X32, 64X64, 4X8, 8X4, 8X16, 16X8, 16X32, 32X16, 32X64, 64X32,
    #           4X16, 16X4, 8X32, 32X8, 16X64, 64X16
    tr = lambda v, w, h: v.reshape(h, w).T.ravel()  # noqa: E731  (transpose of an h-row, w-column matrix)
    for i in range(15):
        for j in range(2):
            m = {}
            m[5], m[6] = t84[i, j], tr(t84[i, j], 8, 4)
            m[13], m[14] = t164[i, j], tr(t164[i, j], 16, 4)
            m[7], m[8] = t168[i, j], tr(t168[i, j], 16, 8)
            m[15], m[16] = t328[i, j], tr(t328[i, j], 32, 8)
            m[9], m[10] = t3216[i, j], tr(t3216[i, j], 32, 16)
            m[0] = untri(t44[i, j], 4)
            m[1] = untri(t88[i, j], 8)
            m[3] = untri(t3232[i, j], 32)
            m[2] = m[3].reshape(32, 32)[::2, ::2].ravel()
            m[4], m[12], m[18], m[11], m[17] = m[3], m[3], m[10], m[3], m[9]
            for tx in range(19):
                emit(lines, f"k_qm_{i}_{j}_{tx}", m[tx], "uint8_t")


def main(src):
    os.makedirs(OUT, exist_ok=True)
    for fname, fn in [("cdf_default.inc", gen_cdf), ("scan.inc", gen_scan), ("dq.inc", gen_dq),
                      ("qm.inc", gen_qm)]:
        lines = [f"/* {fname}: AV1 normative data, generated by tools/gen_dec_tables.py — do not edit */"]
        fn(src, lines)
        with open(os.path.join(OUT, fname), "w") as f:
            f.write("\n".join(lines) + "\n")
        print(fname, len(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src")
