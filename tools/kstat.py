"""Per-kernel static stats from a gfx950 .s file: VALU/SALU/LDS/VMEM counts,
s_nop wait cycles, VGPR/SGPR counts (dev tool)."""
import re
import subprocess
import sys


def stats(path, filt=""):
    txt = open(path).read()
    out = []
    for m in re.finditer(r"^(\S+):\s*;\s*@\S+\n(.*?)s_endpgm", txt, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if filt and filt not in name:
            continue
        valu = len(re.findall(r"^\s+v_", body, re.M))
        salu = len(re.findall(r"^\s+s_(?!nop)", body, re.M))
        nopc = sum(int(x) + 1 for x in re.findall(r"^\s+s_nop (\d+)", body, re.M))
        lds = len(re.findall(r"^\s+ds_", body, re.M))
        mov = len(re.findall(r"^\s+v_mov_b32", body, re.M))
        md = re.search(r"\.name:\s+%s\b.*?\.vgpr_count:\s+(\d+)" % re.escape(name), txt, re.S)
        sg = re.search(r"\.name:\s+%s\b.*?\.sgpr_count:\s+(\d+)" % re.escape(name), txt, re.S)
        demangled = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        out.append((demangled[:70], valu, mov, nopc, salu, lds, md.group(1) if md else "?", sg.group(1) if sg else "?"))
    return out


if __name__ == "__main__":
    for r in stats(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print("%-70s VALU %5d mov %4d nopcyc %4d SALU %4d LDS %3d vgpr %s sgpr %s" % r)
