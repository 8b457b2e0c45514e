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
read's register (source or destination) is a hazard. The pending state flows over the kernel's control-flow
graph (fall-through, forward and backward branch targets; a join takes the union of its predecessors'
pending reads) to a fixed point, so a hazard on a taken forward branch or around a loop back edge is seen.

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


MAX_PENDING = 16  # the lgkm counter saturates: the wave stalls rather than keep more LDS operations in flight


def merge(a, b):
    """Join of two pending lists (oldest first) at a control-flow merge: aligned from the youngest entry, each
    position holds the union of both paths' registers (conservative for any later lgkmcnt(N))."""
    if a is None:
        return b
    n = max(len(a), len(b))
    a = (frozenset(),) * (n - len(a)) + a
    b = (frozenset(),) * (n - len(b)) + b
    return tuple(x | y for x, y in zip(a, b))


def step(ins, pending):
    """Transfer one instruction: (new pending tuple, registers it touched while pending, or empty)."""
    op = ins.split()[0] if ins else ""
    if op == "s_waitcnt":
        m = LGKM.search(ins)
        if m:
            n = int(m.group(1))
            pending = pending[len(pending) - n:] if 0 < n < len(pending) else (() if n == 0 else pending)
        return pending, set()
    touched = regs(ins)
    live = set().union(*pending) if pending else set()
    if op.startswith("ds_"):
        dst = regs(ins[len(op):].split(",")[0]) if op.startswith("ds_read") else set()
        srcs = touched - dst if op.startswith("ds_read") else touched
        return (pending + (frozenset(dst),))[-MAX_PENDING:], srcs & live  # a pending dst may be re-read into
    return pending, touched & live


def successors(i, ins, base, addr_index, n):
    op = ins.split()[0] if ins else ""
    out = []
    if op.startswith("s_cbranch") or op == "s_branch":
        t = TARGET.search(ins)
        if t:
            j = addr_index.get(base + int(t.group(2), 16))
            if j is not None:
                out.append(j)
    if op not in ("s_branch", "s_endpgm", "s_setpc_b64") and i + 1 < n:
        out.append(i + 1)
    return out


def check_kernel(base, insns):
    """Hazards of one kernel: a worklist dataflow over the control-flow graph (fall-through, forward and
    backward branch targets), the pending list at a join being the merge of its predecessors'."""
    n = len(insns)
    if not n:
        return []
    addr_index = {a - 0: i for i, (a, _) in enumerate(insns)}
    state = [None] * n
    state[0] = ()
    work, hz = [0], {}
    while work:
        i = work.pop()
        out, bad = step(insns[i][1], state[i])
        if bad:
            hz[insns[i][0]] = (insns[i][0], insns[i][1], sorted(bad))
        for j in successors(i, insns[i][1], base, addr_index, n):
            m = merge(state[j], out)
            if m != state[j]:
                state[j] = m
                work.append(j)
    return [hz[a] for a in sorted(hz)]


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
