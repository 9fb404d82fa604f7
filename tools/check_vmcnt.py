"""Static check of every kernel's vector-memory waits (the producers of
k_gcn_fwd_pc issue their prefetch loads through inline asm and wait with hand-written
`s_waitcnt vmcnt(n)`; the compiler regards an asm output register as valid when the asm
statement ends, so a copy it placed before the wait would read a register whose load is still
in flight, and nothing would diagnose it).

The check runs on the gfx950 code object itself (disassembled with llvm-objdump), so it sees
the schedule the compiler actually emitted.  Per kernel, a forward dataflow over the control-
flow graph tracks the vector-memory operations in flight, youngest first: every buffer_ /
global_ / flat_ / scratch_ operation enters the queue (on gfx9 `vmcnt` counts loads, stores
and atomics, and they retire in order), with the VGPRs a load (or returning atomic) writes;
`s_waitcnt vmcnt(n)` keeps the n youngest.  At a join the queues are merged position by
position (union), so a register counts as in flight if it is on ANY path.  Any instruction
other than a later load's own destination that names a VGPR of a load still in flight --
reading it, or overwriting it before the load lands -- is reported.

  python tools/check_vmcnt.py leak-det-gnn_amd/build/gcn_nm.o [--kernel k_gcn_fwd_pc]

Exit status 1 when any kernel has a violation.  tests/test_host.py runs it on every object.
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_FUNC = re.compile(r"^[0-9a-f]+ <(\S+)>:$")
_INS = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
_TGT = re.compile(r"<(\S+)\+0x([0-9a-f]+)>\s*$")
_VRANGE = re.compile(r"(?<![\w\[])v\[(\d+):(\d+)\]")
_VONE = re.compile(r"(?<![\w\[])v(\d+)\b")
_VMEM = ("buffer_", "global_", "flat_", "scratch_")
_STOP = ("s_endpgm", "s_setpc_b64", "s_trap", "s_endpgm_saved")
MAXQ = 64
# kernels checked under check_kernel's full_exec assumption (their waves run with all lanes)
FULL_EXEC = ("k_gcn_fwd_pc",)


def disassemble(obj: Path) -> str:
    """gfx950 disassembly of a host object / shared library with an embedded offload bundle,
    or of a bare gfx950 ELF."""
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        elf = obj
        if subprocess.run([str(LLVM / "llvm-readelf"), "-S", str(obj)], capture_output=True,
                          text=True).stdout.find(".hip_fatbin") >= 0:
            fat = d / "fatbin.bin"
            subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(obj), str(d / "x")],
                           check=True, capture_output=True)
            elf = d / "gfx950.elf"
            subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                            f"--targets={TARGET}", f"--output={elf}"], check=True, capture_output=True)
        return subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(elf)], check=True,
                              capture_output=True, text=True).stdout


def vregs(text: str) -> set:
    out = set()
    for a, b in _VRANGE.findall(text):
        out.update(range(int(a), int(b) + 1))
    for a in _VONE.findall(_VRANGE.sub("", text)):
        out.add(int(a))
    return out


def parse(dis: str) -> dict:
    """kernel name -> list of (addr, mnemonic, operands, branch target addr or None)"""
    funcs, cur, base = {}, None, 0
    for line in dis.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = m.group(1)
            base = int(line.split()[0], 16)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = _INS.match(line)
        if not m:
            continue
        mn, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        tgt = None
        if mn.startswith(("s_branch", "s_cbranch")):
            t = _TGT.search(line)
            if t and t.group(1) == cur:
                tgt = base + int(t.group(2), 16)
        funcs[cur].append((addr, mn, ops, tgt))
    return funcs


def _vm_entry(mn: str, ops: str):
    """(is a vector-memory op, VGPRs it writes when it lands)"""
    if not mn.startswith(_VMEM):
        return False, frozenset()
    first = ops.split(",")[0] if ops else ""
    if "_load" in mn and " lds" not in f" {ops} ":
        return True, frozenset(vregs(first))
    if "_atomic" in mn and re.search(r"\b(sc0|glc)\b", ops):
        return True, frozenset(vregs(first))
    return True, frozenset()


# what a register copy or spill looks like (check_kernel's copies_only mode)
_COPY = ("v_mov", "v_accvgpr", "v_cndmask", "v_readlane", "v_readfirstlane", "scratch_store", "buffer_store",
         "global_store")


def check_kernel(ins: list, full_exec: bool = False, copies_only: bool = False) -> list:
    """Violations [(addr, text, regs)] of one kernel.  full_exec: the kernel's waves never reach
    an `s_cbranch_execz` with no lane active, so its skip edge is not followed (k_gcn_fwd_pc:
    the producer and consumer bodies run with all 64 lanes; the compiler still guards them with
    execz skips, and a skip over a refill's loads is the one path that would shift the explicit
    vmcnt counts).  copies_only: report only copies and spills of an in-flight register (the
    failure ADVICE r05 names: a move, select or spill the compiler placed before the hand-written
    wait reading the register; a register the compiler itself redefines is no longer tracked).  The
    unrolled, jump-threaded producer loop of k_gcn_fwd_pc has paths in its CFG that no execution
    takes (a refill followed by the same buffer's wait without the other buffer's step, through
    branches on the same tile compare), and the path-insensitive merge reports the buffer's
    arithmetic on them; a real read before the wait would also fail every parity test."""
    if not ins:
        return []
    idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    starts = {0}
    for i, (a, mn, ops, tgt) in enumerate(ins):
        if tgt is not None and tgt in idx:
            starts.add(idx[tgt])
        if mn.startswith(("s_branch", "s_cbranch")) or mn in _STOP:
            starts.add(i + 1)
    starts = sorted(s for s in starts if s < len(ins))
    block_of = {}
    blocks = []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(ins)
        block_of[s] = k
        blocks.append((s, e))
    succ = []
    for s, e in blocks:
        a, mn, ops, tgt = ins[e - 1]
        out = []
        if tgt is not None and tgt in idx and not (full_exec and mn == "s_cbranch_execz"):
            out.append(block_of[idx[tgt]])
        if not (mn.startswith("s_branch") or mn in _STOP) and e < len(ins):
            out.append(block_of[e])
        succ.append(out)

    def join(p, q):
        n = max(len(p), len(q))
        return tuple((p[i] if i < len(p) else frozenset()) | (q[i] if i < len(q) else frozenset()) for i in range(n))

    state_in = {0: ()}
    work = [0]
    viol = {}
    while work:
        b = work.pop()
        st = list(state_in[b])
        s, e = blocks[b]
        for i in range(s, e):
            a, mn, ops, _ = ins[i]
            if mn == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", ops)
                if m:
                    st = st[:int(m.group(1))]
                continue
            is_vm, dest = _vm_entry(mn, ops)
            pend = set().union(*st) if st else set()
            used = vregs(ops)
            if is_vm and dest:
                used -= dest  # a later load overwriting an older one's register lands after it (in order)
            if copies_only and not is_vm and mn.startswith("v_") and ops:
                parts = ops.split(",", 1)
                wr, rd = vregs(parts[0]), vregs(parts[1]) if len(parts) > 1 else set()
                bad = (rd & pend) if mn.startswith(_COPY) else set()
                if wr & pend:  # the path-insensitive merge: the compiler's own def ends the register's load
                    st = [e - frozenset(wr) for e in st]
            else:
                bad = used & pend
                if copies_only and not mn.startswith(_COPY):
                    bad = set()
            if bad:
                viol[a] = (f"{mn} {ops}", sorted(bad))
            if is_vm:
                st = ([dest] + st)[:MAXQ]
        out = tuple(st)
        for nb in succ[b]:
            old = state_in.get(nb)
            new = out if old is None else join(old, out)
            if new != old:
                state_in[nb] = new
                work.append(nb)
    return [(a, t, r) for a, (t, r) in sorted(viol.items())]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("objects", nargs="+")
    ap.add_argument("--kernel", default="", help="only kernels whose name contains this")
    args = ap.parse_args(argv)
    bad = 0
    for obj in args.objects:
        funcs = parse(disassemble(Path(obj)))
        for name, ins in funcs.items():
            if args.kernel and args.kernel not in name:
                continue
            full = any(k in name for k in FULL_EXEC)
            v = check_kernel(ins, full_exec=full, copies_only=full)
            if v:
                bad += 1
                print(f"{obj}: {name}: {len(v)} instruction(s) use a VGPR whose load is in flight")
                for a, t, r in v[:5]:
                    print(f"    {a:#x}: {t}   regs {r}")
        print(f"{obj}: {sum(1 for n in funcs if args.kernel in n)} kernel(s) checked")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
