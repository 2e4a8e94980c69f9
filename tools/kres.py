"""Dev tool: per-kernel resources of a built HIP library (VGPRs, spills,
scratch, LDS, code size), read from the gfx950 code objects' metadata notes.
Used to check that a kernel edit did not tip the register allocator
(k_pcompress is register-allocation bound).
    usage: python tools/kres.py [lib.so] [kernel-substring]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat")
        subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat])
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            part = os.path.join(d, f"b{i}")
            open(part, "wb").write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, f"co{i}")
            subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                   "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
            yield open(co, "rb").read()


def kernels(lib):
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(code_objects(lib)):
            p = os.path.join(d, f"co{i}")
            open(p, "wb").write(co)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", p], capture_output=True, text=True).stdout
            syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "--wide", p], capture_output=True, text=True).stdout
            sizes = {}
            for line in syms.splitlines():
                f = line.split()
                if len(f) == 8 and f[3] == "FUNC":
                    sizes[f[7]] = int(f[2])
            for blk in notes.split("  - .agpr_count")[1:]:
                def g(k):
                    m = re.search(r"\.%s:\s+(\S+)" % re.escape(k), blk)
                    return m.group(1) if m else None
                name = g("name")
                out[name] = {k: g(k) for k in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "sgpr_spill_count",
                                               "private_segment_fixed_size", "group_segment_fixed_size")}
                dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
                out[name]["demangled"] = dem
                out[name]["code_bytes"] = sizes.get(name)
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else "dietgpu_fork_amd/_lib/libdietgpu_amd.so"
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, r in sorted(kernels(lib).items(), key=lambda kv: kv[1]["demangled"]):
        if filt in r["demangled"]:
            print(f"{r['demangled'][:90]:90s} vgpr {r['vgpr_count']:>4} vspill {r['vgpr_spill_count']:>3} "
                  f"sgpr {r['sgpr_count']:>3} sspill {r['sgpr_spill_count']:>3} scratch "
                  f"{r['private_segment_fixed_size']:>4} lds {r['group_segment_fixed_size']:>6} code {r['code_bytes']}")
