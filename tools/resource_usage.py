"""Per-kernel register / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage output.
usage: python tools/resource_usage.py remarks.txt [name-filter]"""
import re
import subprocess
import sys


def parse(path):
    cur, rec, out = None, {}, []
    for line in open(path):
        m = re.search(r'Function Name: (\S+)', line)
        if m:
            if cur:
                out.append((cur, rec))
            cur, rec = m.group(1), {}
            continue
        m = re.search(r'remark:\s+(\S[^:]*): (\S+) \[-Rpass', line)
        if m and cur:
            rec[m.group(1)] = m.group(2)
    if cur:
        out.append((cur, rec))
    return out


def main():
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, r in parse(sys.argv[1]):
        dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dn = dn.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if flt in dn:
            print(f"{dn:40s} vgpr {r.get('VGPRs')} agpr {r.get('AGPRs')} sgpr {r.get('TotalSGPRs')} "
                  f"scratch {r.get('ScratchSize [bytes/lane]')} occ {r.get('Occupancy [waves/SIMD]')} "
                  f"lds {r.get('LDS Size [bytes/block]')} spill {r.get('SGPRs Spill')}/{r.get('VGPRs Spill')}")


if __name__ == "__main__":
    main()
