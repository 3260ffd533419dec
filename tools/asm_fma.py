"""Per-kernel instruction counts from a device assembly listing (hipcc -S
--offload-device-only): v_fma_f64 (FMA contraction), scratch use and VGPR counts --
the check that the exact stages (md_exact, the 5pt / 7pt root stages) compile without
FMA.  usage: python tools/asm_fma.py kernels_gfx950.s [substring ...]"""
import re
import subprocess
import sys


def main(path, keys):
    s = open(path).read()
    pat = re.compile(r'^(_Z\S+):\s*;', re.M)
    ms = list(pat.finditer(s))
    for i, m in enumerate(ms):
        body = s[m.start(): ms[i + 1].start() if i + 1 < len(ms) else len(s)]
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        if keys and not any(k in name for k in keys):
            continue
        vg = re.search(r'\.amdhsa_next_free_vgpr (\d+)', body)
        sc = re.search(r'\.amdhsa_private_segment_fixed_size (\d+)', body)
        print(f"{name[:100]:100s} fma_f64 {body.count('v_fma_f64'):5d}  vgpr {vg.group(1) if vg else '?':>4s}"
              f"  scratch {sc.group(1) if sc else '?'}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
