"""Check hand-counted LDS waits in a gfx950 code object: no instruction may touch the destination
registers of a `ds_read` before an `s_waitcnt lgkmcnt` has retired that read.

The GEMM kernels issue their LDS fragment reads through inline asm (csrc/kernels/gemm_w4.hip h_read)
and place `s_waitcnt lgkmcnt(N)` themselves, so the compiler believes an asm read's registers hold
data the moment the asm statement issues. If the allocator copies or spills such a register before
the wait (it did: `ds_read_b128 v[0:3]` followed at once by `scratch_store_dwordx4 off, v[0:3]` in
the bias / GELU epilogue instantiations of gemm_w4), the copy takes stale bytes. This scan finds it.

Model: LDS operations complete in order (ds_* only; scalar loads also count in lgkmcnt, which makes
`lgkmcnt(N)` retire at least the reads this model retires, so the check stays conservative).
`lgkmcnt(N)` leaves the N youngest ds operations pending. Any other instruction that names a pending
read's register (source or destination) is a hazard. The scan walks each kernel in address order
(nothing pending after an unconditional branch) and again from every backward-branch target with the
state at the branch (the loop back edge).

  python tools/isa_lds_hazard.py build/obj/gemm_w4.hip.o [kernel-substring]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")
LGKM = re.compile(r"lgkmcnt\((\d+)\)")


def regs(text):
    out = set()
    for kind, lo, hi, one in REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def disassemble(obj):
    """Disassembly text of the gfx950 code object inside a hipcc -c object (offload bundle)."""
    with tempfile.TemporaryDirectory() as d:
        local = os.path.join(d, os.path.basename(obj))
        with open(obj, "rb") as f, open(local, "wb") as g:
            g.write(f.read())
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", local], cwd=d, check=True,
                       capture_output=True)
        cos = [os.path.join(d, n) for n in os.listdir(d) if "gfx950" in n]
        if not cos:
            raise RuntimeError("no gfx950 code object in %s" % obj)
        r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", cos[0]],
                           check=True, capture_output=True, text=True)
        return r.stdout


def kernels(text):
    """{symbol: [(address, instruction text)]}"""
    out, cur, base = {}, None, 0
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            cur, base = m.group(2), int(m.group(1), 16)
            out[cur] = (base, [])
            continue
        if cur is None or not line.startswith("\t"):
            continue
        a = ADDR.search(line)
        if a:
            t = TARGET.search(line)  # branch target, printed in the comment
            out[cur][1].append((int(a.group(1), 16), line.split("//")[0].strip() + (" " + t.group(0) if t else "")))
    return out


def scan(insns, start, state, stop=None):
    """Walk from index `start` with pending list `state`; returns (hazards, {index: state} at backward
    branches)."""
    pending = list(state)
    hazards, back = [], {}
    addr_index = {a: i for i, (a, _) in enumerate(insns)}
    for i in range(start, len(insns)):
        if stop is not None and i == stop:
            break
        addr, ins = insns[i]
        op = ins.split()[0] if ins else ""
        if op == "s_waitcnt":
            m = LGKM.search(ins)
            if m:
                n = int(m.group(1))
                pending = pending[len(pending) - n:] if n < len(pending) else pending
                if n == 0:
                    pending = []
            continue
        touched = regs(ins)
        live = set().union(*pending) if pending else set()
        if op.startswith("ds_"):
            operands = ins[len(op):]
            dst = regs(operands.split(",")[0]) if op.startswith("ds_read") else set()
            srcs = touched - dst if op.startswith("ds_read") else touched
            if srcs & live:  # a pending destination may be re-read into (LDS returns in order)
                hazards.append((addr, ins, sorted(srcs & live)))
            pending.append(frozenset(dst))
            continue
        if touched & live:
            hazards.append((addr, ins, sorted(touched & live)))
        if op.startswith("s_cbranch") or op == "s_branch":
            t = TARGET.search(ins)
            if t:
                tgt = t.group(2)
                back[i] = (tgt, list(pending))
            if op == "s_branch":  # the next instruction is reached from elsewhere: state unknown
                pending = []
        elif op in ("s_endpgm", "s_setpc_b64"):
            pending = []
    return hazards, back, addr_index


def check_kernel(base, insns):
    hazards, back, addr_index = scan(insns, 0, [])
    for i, (off, st) in back.items():
        tgt = base + int(off, 16)
        j = addr_index.get(tgt)
        if j is not None and j <= i and st:
            h2, _, _ = scan(insns, j, st, stop=i + 1)
            hazards += h2
    seen, out = set(), []
    for h in hazards:
        if h[0] not in seen:
            seen.add(h[0])
            out.append(h)
    return out


def check_object(obj, name_filter=""):
    """[(kernel, [(address, instruction, registers)])] for every kernel with a hazard."""
    bad = []
    for name, (base, insns) in kernels(disassemble(obj)).items():
        if name_filter and name_filter not in name:
            continue
        h = check_kernel(base, insns)
        if h:
            bad.append((name, h))
    return bad


def main():
    obj = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    bad = check_object(obj, flt)
    for name, hz in bad:
        print("%s: %d hazards" % (name, len(hz)))
        for addr, ins, rs in hz[:8]:
            print("  %08x  %-60s %s" % (addr, ins[:60], ["%s%d" % r for r in rs[:4]]))
    print("kernels with LDS-read hazards: %d" % len(bad))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
