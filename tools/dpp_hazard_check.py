"""Static check of the gfx950 DPP source hazard in a built libmlhip.so.

The two-lane SHA-256 (transcript_dev.hpp, sha2l_rounds) issues one DPP add
from inline asm (`v_add_u32_dpp ... row_half_mirror ... bank_mask:0x5`).  The
compiler's hazard recognizer does not look inside inline asm, and gfx950
needs 2 wait states between a VALU write of a VGPR and a DPP read of it; the
code passes a register written rounds earlier, and this check proves it for
the code the compiler actually emitted: every DPP instruction of every kernel
is found in the disassembly of each code object in the library's
.hip_fatbin, and the instructions before it are walked back until 2 wait
states are covered (s_nop N = N + 1, any other instruction 1).

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


def check_listing(lines):
    """(dpp instructions checked, [hazard descriptions]) for one disassembly."""
    func, body, checked, bad = None, [], 0, []
    for raw in lines + ["<end>:"]:
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", raw.strip())
        if m or raw == "<end>:":
            func, body = (m.group(1) if m else None), []
            continue
        ins = raw.split("//")[0].strip()
        if not ins or func is None:
            continue
        body.append(ins)
        if "_dpp" not in ins.split()[0]:
            continue
        ops = ins.split(None, 1)[1].split(",") if " " in ins else []
        if len(ops) < 2:
            continue
        src0 = vregs(ops[1].split()[0])
        if not src0:
            continue
        checked += 1
        ws = 0
        for prev in reversed(body[:-1]):
            if ws >= 2:
                break
            op = prev.split()[0]
            mn = re.match(r"s_nop\s+(\S+)", prev)
            if mn:
                ws += int(mn.group(1), 0) + 1
                continue
            if op.startswith("v_") and " " in prev:
                dst = vregs(prev.split(None, 1)[1].split(",")[0])
                if dst & src0:
                    bad.append("%s: '%s' then '%s' (%d wait states)" % (func, prev, ins, ws))
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
