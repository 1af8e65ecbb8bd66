"""Per-kernel register / scratch / LDS usage from `make -C distributed_raytracer_amd/csrc asm`
remarks (-Rpass-analysis=kernel-resource-usage).

usage: make -C distributed_raytracer_amd/csrc asm 2> /tmp/asm.log; python tools/resource_usage.py /tmp/asm.log
"""
import re
import sys


def main(path):
    rows, cur = [], None
    for line in open(path):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/\w+\])?: (\S+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    keys = ["VGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize", "Occupancy", "LDS Size"]
    for r in rows:
        n = re.sub(r"NS_9FrameArgs.*|NS_\d+\w+E$", "", r["name"].replace("_ZN4mirt", ""))
        print(f"{n:40s}", "  ".join(f"{k.split()[0][:5]}{'-sp' if 'Spill' in k else ''}={r.get(k, '?')}" for k in keys))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/asm.log")
