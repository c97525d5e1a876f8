"""Static check of the gfx950 DPP source hazard in a built libmlhip.so.

The two-lane SHA-256 (transcript_dev.hpp, sha2l_rounds) issues one DPP add
from inline asm (`v_add_u32_dpp ... row_half_mirror ... bank_mask:0x5`).  The
compiler's hazard recognizer does not look inside inline asm, and gfx950
needs 2 wait states between a VALU write of a VGPR and a DPP read of it; the
code passes a register written rounds earlier, and this check proves it for
the code the compiler actually emitted: every DPP instruction of every kernel
is found in the disassembly of each code object in the library's
.hip_fatbin, and the instructions before it are walked back until 2 wait
states (VGPR source) and 5 (a VALU write of EXEC) are covered (s_nop N =
N + 1, any other instruction 1).  A block entry whose other predecessors the
listing does not show (function entry, branch target, call return) stops
the walk and must already be covered.

Run on the build host (no GPU):  python tools/dpp_hazard_check.py [lib.so]
Exit status 1 (and the offending instructions) on a hazard."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib, tmp):
    """The gfx950 code objects of every offload bundle in lib's .hip_fatbin."""
    fat = os.path.join(tmp, "fatbin")
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, lib],
                          stderr=subprocess.DEVNULL)
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    out = []
    for i in range(len(offs) - 1):
        b = os.path.join(tmp, "b%d" % i)
        with open(b, "wb") as f:
            f.write(data[offs[i]:offs[i + 1]])
        co = os.path.join(tmp, "co%d" % i)
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--input=" + b, "--targets=" + TARGET, "--output=" + co])
        out.append(co)
    return out


_VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def vregs(tok):
    m = _VREG.match(tok.strip().rstrip(","))
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<(.+)\+0x([0-9a-f]+)>")
_EXEC = ("exec", "exec_lo", "exec_hi")
# 2 wait states between a VALU write of a VGPR and a DPP read of it; 5 between
# a VALU write of EXEC and any DPP (gfx9 rules)
WS_VGPR, WS_EXEC = 2, 5


def _addr(raw):
    m = _ADDR.search(raw)
    return int(m.group(1), 16) if m else None


def _writes_exec(ins):
    op = ins.split()[0]
    if not op.startswith("v_"):
        return False
    if op.startswith("v_cmpx"):
        return True
    rest = ins.split(None, 1)[1] if " " in ins else ""
    return rest.split(",")[0].strip() in _EXEC


def _parse(lines):
    """[(func, base, [(addr, ins, raw)])] from an llvm-objdump listing."""
    funcs, cur = [], None
    for raw in lines:
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", raw.strip())
        if m:
            cur = (m.group(2), int(m.group(1), 16), [])
            funcs.append(cur)
            continue
        ins = raw.split("//")[0].strip()
        if not ins or cur is None:
            continue
        cur[2].append((_addr(raw), ins, raw))
    return funcs


def _entries(func, base, body):
    """Indices in body whose predecessors are not only the listing's previous
    instruction: the function's first instruction (its callers), branch
    targets, and the instruction after a call (the callee returns there)."""
    out = {0}
    addr_ix = {a: i for i, (a, _, _) in enumerate(body) if a is not None}
    for i, (_, ins, raw) in enumerate(body):
        op = ins.split()[0]
        if op.startswith(("s_branch", "s_cbranch")):
            m = _TARGET.search(raw)
            if m and m.group(1) == func and base + int(m.group(2), 16) in addr_ix:
                out.add(addr_ix[base + int(m.group(2), 16)])
            elif not m:
                return None  # a target the listing does not name: unknown everywhere
        elif op.startswith(("s_swappc", "s_call")) and i + 1 < len(body):
            out.add(i + 1)
    return out


def check_listing(lines):
    """(dpp instructions checked, [hazard descriptions]) for one disassembly.

    Walk back from each DPP through the listing.  A block entry with
    predecessors the walk cannot see -- the function's first instruction (its
    callers), a branch target, the instruction after a call (the callee's
    last instructions) -- ends the walk: unless the wait states are already
    covered there, it is reported (put an explicit s_nop before the DPP).
    EXEC writes by VALU (v_cmpx, or a VALU with an exec destination) need 5
    wait states; at an unknown predecessor that rule is reported only when
    the listing holds a VALU EXEC write anywhere (else no path can carry one)."""
    funcs = _parse(lines)
    any_exec = any(_writes_exec(ins) for _, _, body in funcs for _, ins, _ in body)
    checked, bad = 0, []
    for func, base, body in funcs:
        entries = _entries(func, base, body)
        if entries is None:
            entries = set(range(len(body)))
        for i, (_, ins, _) in enumerate(body):
            if "_dpp" not in ins.split()[0]:
                continue
            ops = ins.split(None, 1)[1].split(",") if " " in ins else []
            if len(ops) < 2:
                continue
            src0 = vregs(ops[1].split()[0])
            if not src0:
                continue
            checked += 1
            ws, j = 0, i
            while ws < WS_EXEC:
                if j in entries:  # predecessors of body[j] other than body[j-1] are unseen
                    if ws < WS_VGPR:
                        bad.append("%s: '%s' %d wait states after a block entry with unseen "
                                   "predecessors ('%s')" % (func, ins, ws, body[j][1]))
                    elif any_exec:
                        bad.append("%s: '%s' %d wait states after a block entry; a VALU EXEC "
                                   "write may precede it" % (func, ins, ws))
                    break
                j -= 1
                prev = body[j][1]
                mn = re.match(r"s_nop\s+(\S+)", prev)
                if mn:
                    ws += int(mn.group(1), 0) + 1
                    continue
                if prev.split()[0].startswith("v_") and " " in prev:
                    if ws < WS_VGPR and vregs(prev.split(None, 1)[1].split(",")[0]) & src0:
                        bad.append("%s: '%s' then '%s' (%d wait states)" % (func, prev, ins, ws))
                        break
                    if _writes_exec(prev):
                        bad.append("%s: EXEC write '%s' then '%s' (%d wait states)" % (func, prev, ins, ws))
                        break
                ws += 1
    return checked, bad


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    lib = argv[0] if argv else os.path.join(ROOT, "multilinear_amd", "libmlhip.so")
    total, bad = 0, []
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co],
                                 check=True, capture_output=True, text=True).stdout.splitlines()
            c, b = check_listing(dis)
            total += c
            bad += b
    print("dpp_hazard_check: %d DPP instructions checked, %d hazards" % (total, len(bad)))
    for b in bad[:20]:
        print("  " + b)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
