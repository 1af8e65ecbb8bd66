"""Per-kernel registers, spills, scratch and LDS straight from a built libmirt.so's code-object
metadata (no asm build): python tools/co_usage.py [lib.so] [name-filter]"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    from test_kernarg_layout import _code_object, _kernels
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else os.path.join(ROOT, "distributed_raytracer_amd", "libmirt.so")
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for k in sorted(_kernels(_code_object(lib)), key=lambda k: k[".name"]):
        n = re.sub(r"EEEv.*|Ev.*", "", k[".name"].replace("_ZN4mirt", ""))
        if flt not in n:
            continue
        print(f"{n:44s} vgpr={k['.vgpr_count']:3d} vsp={k['.vgpr_spill_count']:3d} sgpr={k['.sgpr_count']:3d} "
              f"ssp={k['.sgpr_spill_count']:3d} scratch={k['.private_segment_fixed_size']:3d} "
              f"lds={k['.group_segment_fixed_size']}")


if __name__ == "__main__":
    main()
