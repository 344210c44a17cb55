"""Register / scratch / LDS / occupancy of every production kernel, from the
compiler (hipcc -Rpass-analysis=kernel-resource-usage, the _build.py flags),
plus scratch_insts: the scratch / private-buffer load and store instructions
actually present in each kernel's ISA (ScratchSize alone is the frame the
compiler reserved, which may have no access left in the code).

    python tools/resource_usage.py [out.json]      (CPU only: hipcc cross-compiles)

DESIGN.md quotes these figures; regenerate them each round
rather than carrying numbers forward.
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "self-play-racing_amd"))
from rx import _build  # noqa: E402

FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "SGPRs": "sgpr", "TotalSGPRs": "sgpr_total",
          "ScratchSize [bytes/lane]": "scratch_bytes_per_lane", "Occupancy [waves/SIMD]": "occupancy_waves_per_simd",
          "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill", "LDS Size [bytes/block]": "lds_bytes_per_block"}


def demangle(name):
    try:
        return subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt", name], capture_output=True, text=True,
                              check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return name


def main():
    out = {}
    tmp = tempfile.mkdtemp(prefix="rxres_")
    for src in _build.SOURCES:
        if not src.endswith(".hip"):
            continue
        cmd = [_build.hipcc()] + _build.FLAGS + ["-c", os.path.join(_build.CSRC, src), "-o",
                                                 os.path.join(tmp, src + ".o"), "-Rpass-analysis=kernel-resource-usage"]
        text = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
        cur = None
        for line in text.splitlines():
            m = re.search(r"remark:\s+Function Name: (\S+)", line)
            if m:
                cur = demangle(m.group(1)).replace("(anonymous namespace)::", "")
                out[cur] = {"source": src}
                continue
            m = re.search(r"remark:\s+([A-Za-z ]+(?:\[[^\]]+\])?): (\d+)", line)
            if m and cur and m.group(1).strip() in FIELDS:
                out[cur][FIELDS[m.group(1).strip()]] = int(m.group(2))
        # the compiler's ScratchSize is the private-segment FRAME, which can be reserved with no
        # scratch access left in the code (measured: most env kernels); count the actual
        # scratch / private-buffer instructions in the kernel's ISA
        asm = os.path.join(tmp, src + ".s")
        cmd_s = [_build.hipcc()] + _build.FLAGS + ["-c", os.path.join(_build.CSRC, src), "--cuda-device-only", "-S",
                                                   "-o", asm]
        subprocess.run(cmd_s, capture_output=True, text=True, check=True)
        cur_sym = None
        ops = {}
        for line in open(asm):
            m = re.match(r"^(_Z\S+):", line)
            if m:
                cur_sym = demangle(m.group(1)).replace("(anonymous namespace)::", "")
                ops.setdefault(cur_sym, 0)
                continue
            if cur_sym and re.search(r"\b(scratch_(load|store)\w*|buffer_(load|store)\w*)\b", line):
                ops[cur_sym] += 1
        for k, n in ops.items():
            if k in out:
                out[k]["scratch_insts"] = n
    s = json.dumps(out, indent=1, sort_keys=True)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(s + "\n")
    for k, v in sorted(out.items()):
        print(f"{k[:70]:70s} vgpr {v.get('vgpr', 0):3d} agpr {v.get('agpr', 0):3d} scratch {v.get('scratch_bytes_per_lane', 0):3d}"
              f" scratch_insts {v.get('scratch_insts', -1):3d}"
              f" sgpr_spill {v.get('sgpr_spill', 0):3d} vgpr_spill {v.get('vgpr_spill', 0):3d} occ {v.get('occupancy_waves_per_simd', 0)}"
              f" lds {v.get('lds_bytes_per_block', 0)}")


if __name__ == "__main__":
    main()
