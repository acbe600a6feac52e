"""Structural checks on the gfx950 code object shipped in rav1d_amd/librav1d_amd.so (test
infrastructure, CPU only).

The one-grid MC hand-off (mi_mc_frame_sync, rav1d_amd/csrc/mc.hip) publishes a SEG mask with
`sc1` word stores, drains them (`s_waitcnt vmcnt(0)`) and then stores one flag per tile; a
waiting wave polls the flags and afterwards reads the mask with `sc1` word loads, without an
acquire. That is correct only while the emitted code keeps three properties, which this module
checks on the disassembly of `mc_kernel`:

1. every `sc1` access is a `global_*` instruction and the kernel holds no `flat_*` access;
2. no mask load can execute before a poll loop has exited: every `sc1` load outside the poll
   loops (the strongly connected parts of the control-flow graph holding `s_sleep`) cannot
   reach a poll loop;
3. every flag store is drained: on every path into a final `sc1` store (one from which no
   other `sc1` store is reachable), the nearest earlier `sc1` store lies behind an
   `s_waitcnt` with `vmcnt(0)`.
"""
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def code_objects(lib_path):
    """The gfx950 code objects (bytes) of a hipcc-linked shared library: one per translation
    unit, each a clang offload bundle inside .hip_fatbin."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib_path,
                        os.path.join(td, "scratch.so")], check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(_MAGIC), data)] + [len(data)]
        out = []
        for k in range(len(starts) - 1):
            bi, co = os.path.join(td, f"b{k}"), os.path.join(td, f"c{k}.co")
            open(bi, "wb").write(data[starts[k]:starts[k + 1]])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            f"--targets={_TARGET}", f"--input={bi}", f"--output={co}"],
                           check=True, capture_output=True)
            out.append(open(co, "rb").read())
        return out


def disassemble(co_bytes):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co_bytes)
        f.flush()
        r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", f.name],
                           check=True, capture_output=True, text=True)
        return r.stdout


_FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:")
_INSN = re.compile(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):")
_TGT = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")


def functions(asm):
    """{symbol: [(addr, text), ...]} in address order."""
    funcs, cur = {}, None
    for line in asm.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = funcs.setdefault(m.group(2), [])
            base = int(m.group(1), 16)
            cur.append(("base", base))
            continue
        m = _INSN.match(line)
        if m and cur is not None:
            text = m.group(1)
            t = _TGT.search(line)
            cur.append((int(m.group(2), 16), text, int(t.group(2), 16) if t else None))
    out = {}
    for name, items in funcs.items():
        base = items[0][1]
        out[name] = [(a, txt, None if off is None else base + off) for (a, txt, off) in items[1:]]
    return out


class Cfg:
    """Basic blocks of one function: blocks[i] = list of instruction texts, succ[i] = [j]."""

    def __init__(self, insns):
        addrs = [a for a, _, _ in insns]
        leaders = {addrs[0]}
        for k, (a, txt, tgt) in enumerate(insns):
            op = txt.split()[0]
            if op.startswith("s_cbranch") or op == "s_branch":
                if tgt is not None:
                    leaders.add(tgt)
                if k + 1 < len(insns):
                    leaders.add(addrs[k + 1])
            elif op in ("s_endpgm", "s_setpc_b64") and k + 1 < len(insns):
                leaders.add(addrs[k + 1])
        starts = sorted(x for x in leaders if x in set(addrs))
        index = {a: i for i, a in enumerate(starts)}
        self.blocks, self.succ = [], []
        pos = {a: k for k, a in enumerate(addrs)}
        for i, s in enumerate(starts):
            end = pos[starts[i + 1]] if i + 1 < len(starts) else len(insns)
            body = insns[pos[s]:end]
            self.blocks.append([t for _, t, _ in body])
            last_op = body[-1][1].split()[0]
            nxt = []
            if last_op == "s_branch":
                nxt.append(index[body[-1][2]])
            elif last_op.startswith("s_cbranch"):
                nxt.append(index[body[-1][2]])
                if i + 1 < len(starts):
                    nxt.append(i + 1)
            elif last_op not in ("s_endpgm", "s_setpc_b64") and i + 1 < len(starts):
                nxt.append(i + 1)
            self.succ.append(nxt)
        self.pred = [[] for _ in self.blocks]
        for i, ss in enumerate(self.succ):
            for j in ss:
                self.pred[j].append(i)

    def reach(self, i):
        """Blocks reachable from block i by one or more edges."""
        seen, stack = set(), list(self.succ[i])
        while stack:
            j = stack.pop()
            if j not in seen:
                seen.add(j)
                stack.extend(self.succ[j])
        return seen


def _is_sc1_load(t):
    return t.startswith(("global_load", "buffer_load")) and re.search(r"\bsc1\b", t) is not None


def _is_sc1_store(t):
    return t.startswith(("global_store", "buffer_store")) and re.search(r"\bsc1\b", t) is not None


def _drains(t):
    return t.startswith("s_waitcnt") and "vmcnt(0)" in t


def check_handoff(insns):
    """Returns a list of violations (empty: the three properties hold) and a summary dict."""
    errs = []
    texts = [t for _, t, _ in insns]
    for t in texts:
        if t.startswith("flat_"):
            errs.append(f"flat access: {t}")
        elif re.search(r"\bsc1\b", t) and not t.startswith(("global_", "buffer_", "s_")):
            errs.append(f"sc1 access that is not global_: {t}")
    g = Cfg(insns)
    n = len(g.blocks)
    reach = [g.reach(i) for i in range(n)]
    # poll loops: blocks on a cycle through a block holding s_sleep
    sleepers = [i for i in range(n) if any(t.startswith("s_sleep") for t in g.blocks[i])]
    loop = set()
    for s in sleepers:
        if s in reach[s]:
            loop |= {j for j in reach[s] if s in reach[j]} | {s}
    mask_loads = [(i, t) for i in range(n) if i not in loop for t in g.blocks[i] if _is_sc1_load(t)]
    poll_loads = [(i, t) for i in loop for t in g.blocks[i] if _is_sc1_load(t)]
    if not loop:
        errs.append("no poll loop (s_sleep on a cycle) found")
    if not poll_loads:
        errs.append("no sc1 load inside the poll loops")
    if not mask_loads:
        errs.append("no sc1 mask load outside the poll loops")
    for i, t in mask_loads:
        if reach[i] & loop:
            errs.append(f"mask load can run before a poll loop: block {i}: {t}")
    # producer: final sc1 stores and the drain before them
    stores = [(i, k) for i in range(n) for k, t in enumerate(g.blocks[i]) if _is_sc1_store(t)]
    store_blocks = {i for i, _ in stores}

    def later_store(i, k):
        if any(_is_sc1_store(t) for t in g.blocks[i][k + 1:]):
            return True
        return bool(reach[i] & store_blocks)

    finals = [(i, k) for i, k in stores if not later_store(i, k)]
    if not finals:
        errs.append("no final sc1 (flag) store found")

    def drained_before(i, k):
        # walk every path backwards from instruction k of block i; stop at a drain; fail at an
        # earlier sc1 store or the function entry
        work, seen = [(i, k)], set()
        while work:
            b, pos = work.pop()
            hit = None
            for t in reversed(g.blocks[b][:pos]):
                if _drains(t):
                    hit = "drain"
                    break
                if _is_sc1_store(t):
                    hit = "store"
                    break
            if hit == "store":
                return False
            if hit == "drain":
                continue
            if not g.pred[b]:
                continue   # the entry: no earlier store on this path
            for p in g.pred[b]:
                if p not in seen:
                    seen.add(p)
                    work.append((p, len(g.blocks[p])))
        return True

    for i, k in finals:
        if not drained_before(i, k):
            errs.append(f"flag store without a vmcnt(0) drain after the mask stores: block {i}: {g.blocks[i][k]}")
    summary = dict(blocks=n, poll_loop_blocks=len(loop), poll_loads=len(poll_loads),
                   mask_loads=len(mask_loads), sc1_stores=len(stores), flag_stores=len(finals))
    return errs, summary
