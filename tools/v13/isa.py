"""Tiny CDNA4 (gfx950) instruction DSL for the generated attn_fwd_v13 body.

An instruction is an `Ins` (opcode, operand list, modifier text).  The same
objects are printed as assembler text (tools/gen_flash_v13.py puts the text
into one inline-asm statement of csrc/flash_v13.hip) and executed by the CPU
emulator (tools/v13/emu.py), so what is tested on the CPU is exactly what the
GPU runs.

`finalize()` is the hazard / wait-count pass that hipcc does not do for an
inline-asm body (cdna_hip_programming.md §5.7): a forward dataflow over the
control-flow graph tracks, per register, the wait states since its last
writer and the memory operations still in flight, and inserts the `s_nop`
padding and the counted `s_waitcnt` each read needs.  The wait-state numbers
are LLVM's for gfx950, read off hipcc's own output for the same instruction
pairs (tools/v13/README: the probe kernels).
"""
from __future__ import annotations

import struct


class Reg:
    """A register or register range: file 'v', 'a', 's', or a special
    ('vcc', 'exec', 'm0', 'scc')."""
    __slots__ = ("f", "i", "n")

    def __init__(self, f, i=0, n=1):
        self.f, self.i, self.n = f, i, n

    def __str__(self):
        if self.f in ("vcc", "exec", "m0", "scc"):
            return self.f
        return f"{self.f}{self.i}" if self.n == 1 else f"{self.f}[{self.i}:{self.i + self.n - 1}]"

    __repr__ = __str__

    def __getitem__(self, k):
        assert 0 <= k < self.n, (self, k)
        return Reg(self.f, self.i + k, 1)

    def sub(self, k, n):
        assert 0 <= k and k + n <= self.n, (self, k, n)
        return Reg(self.f, self.i + k, n)

    def names(self):
        if self.f in ("vcc", "exec"):
            return [self.f]
        if self.f in ("m0", "scc"):
            return [self.f]
        return [f"{self.f}{self.i + k}" for k in range(self.n)]


def V(i, n=1):
    assert 0 <= i and i + n <= 256, (i, n)
    return Reg("v", i, n)


def A(i, n=1):
    assert 0 <= i and i + n <= 256, (i, n)
    return Reg("a", i, n)


def S(i, n=1):
    assert 0 <= i and i + n <= 102, (i, n)
    return Reg("s", i, n)


VCC, EXEC, M0, SCC = Reg("vcc"), Reg("exec"), Reg("m0"), Reg("scc")


class Neg:
    __slots__ = ("r",)

    def __init__(self, r):
        self.r = r

    def __str__(self):
        return f"-{self.r}"


def fbits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


def fmt(o):
    if isinstance(o, (Reg, Neg)):
        return str(o)
    if isinstance(o, bool):
        return str(int(o))
    if isinstance(o, int):
        return str(o) if -16 <= o <= 64 else hex(o & 0xFFFFFFFF)
    if isinstance(o, float):
        return hex(fbits(o))
    return str(o)


class Ins:
    __slots__ = ("op", "ops", "mods", "note")

    def __init__(self, op, *ops, mods="", note=""):
        self.op, self.ops, self.mods, self.note = op, list(ops), mods, note

    def text(self):
        if self.op == "label":
            return f"{self.ops[0]}:"
        s = self.op
        if self.ops:
            s += " " + ", ".join(fmt(o) for o in self.ops)
        if self.mods:
            s += " " + self.mods
        return s

    def __repr__(self):
        return self.text()

    # ---- classification -------------------------------------------------
    def kind(self):
        op = self.op
        if op == "label":
            return "label"
        if op.startswith("v_mfma"):
            return "mfma"
        if op in ("v_exp_f32", "v_rcp_f32", "v_log_f32", "v_sqrt_f32", "v_rsq_f32"):
            return "trans"
        if op.startswith("v_accvgpr_write"):
            return "accw"
        if op.startswith("v_"):
            return "valu"
        if op.startswith("ds_"):
            return "ds"
        if op == "global_load_lds_dwordx4":
            return "dma"
        if op.startswith("global_load"):
            return "vmload"
        if op.startswith("global_store"):
            return "vmstore"
        if op.startswith("s_load") or op in ("s_memtime", "s_memrealtime"):
            return "smem"
        if op in ("s_nop",):
            return "nop"
        if op == "s_waitcnt":
            return "wait"
        if op in ("s_branch", "s_cbranch_scc0", "s_cbranch_scc1", "s_cbranch_vccz", "s_cbranch_vccnz",
                  "s_cbranch_execz"):
            return "branch"
        if op == "s_barrier":
            return "barrier"
        if op == "s_endpgm":
            return "end"
        if op.startswith("s_"):
            return "salu"
        raise ValueError(op)

    def ws(self):
        """wait states this instruction provides to later ones"""
        if self.op == "label":
            return 0
        if self.op == "s_nop":
            return int(self.ops[0]) + 1
        return 1

    def regs_of(self, o):
        if isinstance(o, Neg):
            o = o.r
        return o.names() if isinstance(o, Reg) else []

    def writes(self):
        k, op, o = self.kind(), self.op, self.ops
        if k in ("label", "nop", "wait", "barrier", "branch", "vmstore", "dma", "end"):
            return []
        if op.startswith("v_cmp_") and op.endswith("_e32"):
            return ["vcc"]
        if op.startswith("v_permlane"):
            return self.regs_of(o[0]) + self.regs_of(o[1])
        if op.startswith("s_cmp"):
            return ["scc"]
        w = self.regs_of(o[0])
        if op in ("s_add_u32", "s_sub_u32", "s_addc_u32", "s_subb_u32", "s_and_b32", "s_or_b32",
                  "s_lshl_b32", "s_lshr_b32", "s_and_b64", "s_min_u32", "s_max_u32", "s_add_i32",
                  "s_ashr_i32"):
            w = w + ["scc"]
        if op == "s_and_saveexec_b64":
            w = w + ["exec", "scc"]
        return w

    def reads(self):
        k, op, o = self.kind(), self.op, self.ops
        if k in ("label", "nop", "wait", "barrier", "end"):
            return []
        if k == "branch":
            return {"s_cbranch_scc0": ["scc"], "s_cbranch_scc1": ["scc"], "s_cbranch_vccz": ["vcc"],
                    "s_cbranch_vccnz": ["vcc"], "s_cbranch_execz": ["exec"]}.get(op, [])
        if op == "v_writelane_b32":
            return self.regs_of(o[1]) + self.regs_of(o[0])
        if k in ("vmstore",):
            r = []
            for x in o:
                r += self.regs_of(x)
            return r + ["exec"]
        if k == "dma":
            return self.regs_of(o[0]) + self.regs_of(o[1]) + ["m0", "exec"]
        if op.startswith("v_permlane") or (op.startswith("s_cmp")):
            r = []
            for x in o:
                r += self.regs_of(x)
            return r
        r = []
        for x in o[1:]:
            r += self.regs_of(x)
        if op in ("s_addc_u32", "s_subb_u32", "s_cselect_b32", "s_cselect_b64"):
            r.append("scc")
        if op.startswith("v_cndmask") and op.endswith("_e32"):
            r.append("vcc")
        if op == "s_and_saveexec_b64":
            r.append("exec")
        if k in ("valu", "trans", "accw", "ds", "vmload", "mfma"):
            r.append("exec")
        return r

    def mfma_srcs(self):
        """(srcA names, srcB names, srcC names) of an MFMA"""
        o = self.ops
        return self.regs_of(o[1]), self.regs_of(o[2]), self.regs_of(o[3])


def label(name):
    return Ins("label", name)


def is_waitcnt_text(s):
    return s.startswith("s_waitcnt")


# ---- hazard rules (wait states between a writer and a reader) ------------
# writer class -> reader class -> wait states (LLVM gfx950 numbers from the
# probes: XDL 16x16x32 result -> VALU / VMEM read 8; VALU -> MFMA A/B 2;
# trans -> VALU 1; VALU -> permlane 2; M0 -> LDS-DMA 1; VALU -> DPP source 2,
# LLVM's DppVgprWaitStates)
def need_ws(wcls, rcls):
    if wcls == "mfma":
        return {"valu": 8, "trans": 8, "ds": 8, "vm": 8, "accr": 10, "perm": 8, "dpp": 8, "mfmaAB": 10,
                "mfmaC": 0, "salu": 8, "dma": 8}.get(rcls, 0)
    if wcls == "valu":
        return {"mfmaAB": 2, "mfmaC": 3, "perm": 2, "dpp": 2}.get(rcls, 0)
    if wcls == "trans":
        return {"valu": 1, "trans": 1, "ds": 1, "vm": 1, "perm": 2, "dpp": 2, "mfmaAB": 2, "mfmaC": 3, "accr": 1,
                "dma": 1}.get(rcls, 0)
    if wcls == "accw":
        return {"mfmaAB": 3, "mfmaC": 3, "accr": 1}.get(rcls, 0)
    if wcls == "m0":
        return {"dma": 1, "ds": 1}.get(rcls, 0)
    if wcls == "vsgpr":  # VALU writing an SGPR / VCC
        return {"vm": 5, "smem": 5, "dma": 5, "salu": 0}.get(rcls, 0)
    return 0


def reader_classes(ins):
    """[(regname, reader class)] for every register the instruction reads"""
    k, op = ins.kind(), ins.op
    if k == "mfma":
        a, b, c = ins.mfma_srcs()
        return [(r, "mfmaAB") for r in a + b] + [(r, "mfmaC") for r in c]
    cls = {"valu": "valu", "trans": "trans", "accw": "valu", "ds": "ds", "vmload": "vm", "vmstore": "vm",
           "dma": "dma", "salu": "salu", "smem": "smem", "branch": "salu"}.get(k)
    if cls is None:
        return []
    if op.startswith("v_accvgpr_read"):
        cls = "accr"
    if op.startswith("v_permlane"):
        cls = "perm"
    if op.endswith("_dpp"):
        cls = "dpp"
    return [(r, cls) for r in ins.reads()]


def writer_class(ins, reg):
    k = ins.kind()
    if k == "mfma":
        return "mfma"
    if k == "trans":
        return "trans"
    if k == "accw":
        return "accw"
    if reg == "m0":
        return "m0"
    if k == "valu" and (reg.startswith("s") or reg == "vcc"):
        return "vsgpr"
    if k == "valu":
        return "valu"
    return None


CAP = 24  # wait states beyond any rule


def _succs(prog, i, labels):
    ins = prog[i]
    k = ins.kind()
    if k == "branch":
        t = labels[ins.ops[0]]
        return [t] if ins.op == "s_branch" else [t, i + 1]
    if ins.op == "s_endpgm":
        return []
    return [i + 1] if i + 1 < len(prog) else []


def _merge(a, b):
    """state merge at a join: the worst case of each component"""
    if a is None:
        return b
    ws = dict(a[0])
    for key, d in b[0].items():
        ws[key] = min(d, ws.get(key, CAP))
    srcc = dict(a[1])
    for key, d in b[1].items():
        srcc[key] = min(d, srcc.get(key, CAP))
    lg = dict(a[2])
    for key, d in b[2].items():
        lg[key] = min(d, lg.get(key, 1 << 20))
    vm = dict(a[3])
    for key, d in b[3].items():
        vm[key] = min(d, vm.get(key, 1 << 20))
    return (ws, srcc, lg, vm)


def _eq(a, b):
    return a is not None and b is not None and a[0] == b[0] and a[1] == b[1] and a[2] == b[2] and a[3] == b[3]


def _step(ins, st, fixes, idx):
    """transfer one instruction; record needed fixes (nop wait states and
    waitcnt values) before instruction idx"""
    ws, srcc, lg, vm = dict(st[0]), dict(st[1]), dict(st[2]), dict(st[3])
    k = ins.kind()
    need_nop = 0
    need_lg = None
    need_vm = None
    if k not in ("label", "nop", "wait"):
        for reg, rcls in reader_classes(ins):
            for (r, wc), d in ws.items():
                if r == reg:
                    need_nop = max(need_nop, need_ws(wc, rcls) - d)
            if reg in lg:
                need_lg = lg[reg] if need_lg is None else min(need_lg, lg[reg])
            if reg in vm:
                need_vm = vm[reg] if need_vm is None else min(need_vm, vm[reg])
        for reg in ins.writes():
            if reg in srcc and k in ("valu", "trans", "accw", "ds", "vmload"):
                need_nop = max(need_nop, 4 - srcc[reg])
            if reg in lg:  # WAW with an in-flight load
                need_lg = lg[reg] if need_lg is None else min(need_lg, lg[reg])
            if reg in vm:
                need_vm = vm[reg] if need_vm is None else min(need_vm, vm[reg])
    if need_nop > 0 or need_lg is not None or need_vm is not None:
        f = fixes.setdefault(idx, [0, None, None])
        f[0] = max(f[0], need_nop)
        if need_lg is not None:
            f[1] = need_lg if f[1] is None else min(f[1], need_lg)
        if need_vm is not None:
            f[2] = need_vm if f[2] is None else min(f[2], need_vm)
    # apply the fix's effect to the state so the analysis continues cleanly
    if idx in fixes:
        f = fixes[idx]
        add = f[0]
        if f[1] is not None:
            lg = {r: c for r, c in lg.items() if c < f[1] and f[1] > 0}
        if f[2] is not None:
            vm = {r: c for r, c in vm.items() if c < f[2] and f[2] > 0}
        if add:
            ws = {key: min(CAP, d + add) for key, d in ws.items()}
            srcc = {key: d + add for key, d in srcc.items() if d + add < CAP}
    # effect of the instruction itself
    w = ins.ws()
    if w:
        ws = {key: d + w for key, d in ws.items() if d + w < CAP}
        srcc = {key: d + w for key, d in srcc.items() if d + w < CAP}
    if k == "wait":
        txt = ins.ops[0]
        for part in str(txt).split():
            if part.startswith("lgkmcnt("):
                n = int(part[8:-1])
                lg = {r: c for r, c in lg.items() if c < n and n > 0}
            if part.startswith("vmcnt("):
                n = int(part[6:-1])
                vm = {r: c for r, c in vm.items() if c < n and n > 0}
    if k == "ds" or k == "smem":
        lg = {r: c + 1 for r, c in lg.items()}
        if k == "smem":
            for r in ins.writes():
                lg[r] = -(1 << 20)  # SMEM returns out of order: only lgkmcnt(0) retires it
        elif ins.op.startswith("ds_read"):
            for r in ins.writes():
                lg[r] = 0
    if k in ("vmload", "vmstore", "dma"):
        vm = {r: c + 1 for r, c in vm.items()}
        if k == "vmload":
            for r in ins.writes():
                vm[r] = 0
    for reg in ins.writes():
        ws = {key: d for key, d in ws.items() if key[0] != reg}
        wc = writer_class(ins, reg)
        if wc:
            ws[(reg, wc)] = 0
    if k == "mfma":
        for r in ins.mfma_srcs()[2]:
            srcc[r] = 0
    return (ws, srcc, lg, vm)


def analyse(prog):
    labels = {ins.ops[0]: i for i, ins in enumerate(prog) if ins.op == "label"}
    n = len(prog)
    states = [None] * (n + 1)
    states[0] = ({}, {}, {}, {})
    fixes = {}
    work = [0]
    inq = {0}
    while work:
        i = work.pop()
        inq.discard(i)
        st = _step(prog[i], states[i], fixes, i)
        for j in _succs(prog, i, labels):
            if j >= n:
                continue
            m = _merge(states[j], st)
            if not _eq(m, states[j]):
                states[j] = m
                if j not in inq:
                    inq.add(j)
                    work.append(j)
    return fixes


def finalize(prog, verbose=False):
    """insert the s_nop padding and s_waitcnt each read needs; returns the
    new program and a summary"""
    prog = list(prog)
    total_nops = total_waits = 0
    for _ in range(20):
        fixes = analyse(prog)
        if not fixes:
            break
        out = []
        for i, ins in enumerate(prog):
            f = fixes.get(i)
            if f:
                parts = []
                if f[2] is not None:
                    parts.append(f"vmcnt({max(0, min(63, f[2]))})")
                if f[1] is not None:
                    parts.append(f"lgkmcnt({max(0, min(15, f[1]))})")
                if parts:
                    out.append(Ins("s_waitcnt", " ".join(parts), note="auto"))
                    total_waits += 1
                nn = f[0]
                while nn > 0:
                    q = min(nn, 16)
                    out.append(Ins("s_nop", q - 1, note="auto"))
                    total_nops += q
                    nn -= q
            out.append(ins)
        prog = out
    else:
        raise RuntimeError("hazard pass did not converge")
    if verbose:
        print(f"[v13 finalize] {total_nops} nop wait states, {total_waits} waits")
    return prog, {"nop_ws": total_nops, "waits": total_waits}
