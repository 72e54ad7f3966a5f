"""Per-kernel register, scratch and occupancy table of the shipped gfx950 code
objects, read from their metadata (no GPU needed).

For every build/*.o the Makefile produced, the gfx950 code object is taken out
of the .hip_fatbin offload bundle and its AMDHSA metadata (llvm-readelf
--notes) gives, per kernel: VGPRs (unified arch + acc count, as the wave
allocates them), AGPRs, SGPRs, spills, private segment (scratch) bytes per
lane, LDS bytes and the workgroup size.  Occupancy columns:
  waves/SIMD by registers = min(8, 512 // VGPRs rounded up to 8);
  by LDS = (160 KB // LDS) workgroups per CU x waves per workgroup / 4 SIMDs;
  occupancy = the smaller (at most 8).
Usage: python scripts/kernel_resources.py [out.txt]   (after `make native`)"""
import glob
import os
import subprocess
import sys
import tempfile

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
LDS_PER_CU = 160 * 1024


def code_object(obj, tmp):
    fb = os.path.join(tmp, "fb.bin")
    co = os.path.join(tmp, os.path.basename(obj) + ".co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.devnull],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
    return co


def kernels(co):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    start = notes.index("---")
    end = notes.index("\n...", start)
    meta = yaml.safe_load(notes[start:end])
    return meta.get("amdhsa.kernels", [])


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                         check=True).stdout.splitlines()
    return [o.replace("hhfm::", "").replace("(hhfm::", "(") for o in out]


def occupancy(k):
    vg = max(1, k.get(".vgpr_count", 0))
    by_reg = min(8, 512 // ((vg + 7) // 8 * 8))
    wg = k.get(".max_flat_workgroup_size", 256)
    waves = max(1, (wg + 63) // 64)
    lds = k.get(".group_segment_fixed_size", 0)
    by_lds = 8 if lds == 0 else min(8, (LDS_PER_CU // lds) * waves // 4)
    return by_reg, by_lds, min(by_reg, by_lds)


def main():
    objs = sorted(glob.glob(os.path.join(ROOT, "build", "*.o")))
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            try:
                co = code_object(obj, tmp)
            except subprocess.CalledProcessError:
                continue   # host-only object
            ks = kernels(co)
            names = demangle([k[".name"] for k in ks])
            for k, n in zip(ks, names):
                rows.append((os.path.basename(obj)[:-2], n, k))
    hdr = ("source", "kernel", "VGPR", "AGPR", "SGPR", "vspill", "sspill", "scratchB", "LDS_B",
           "WG", "w/SIMD reg", "w/SIMD lds", "occ")
    lines = ["# gfx950 kernel resources from code-object metadata (scripts/kernel_resources.py)",
             "# VGPR = unified count allocated per wave (arch + acc); scratchB = "
             ".private_segment_fixed_size per lane",
             "\t".join(hdr)]
    nscratch = 0
    for src, n, k in rows:
        r, l, o = occupancy(k)
        scratch = k.get(".private_segment_fixed_size", 0)
        nscratch += scratch > 0
        lines.append("\t".join(str(x) for x in (
            src, n, k.get(".vgpr_count", 0), k.get(".agpr_count", 0), k.get(".sgpr_count", 0),
            k.get(".vgpr_spill_count", 0), k.get(".sgpr_spill_count", 0), scratch,
            k.get(".group_segment_fixed_size", 0), k.get(".max_flat_workgroup_size", 0), r, l,
            o)))
    lines.append(f"# {len(rows)} kernels, {nscratch} with scratch")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(text)
    else:
        sys.stdout.write(text)


if __name__ == "__main__":
    main()
