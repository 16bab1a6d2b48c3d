"""Register / LDS / spill usage of the gfx950 kernels in a hipcc object or shared library: pulls the clang
offload bundle out of the .hip_fatbin section and prints the code object's kernel metadata.
    python tools/kernel_regs.py multimodal-financial-analysis-tool-using-paligemma_amd/csrc/build/kernels_gemm.o [substring]"""
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(path):
    with tempfile.NamedTemporaryFile(suffix=".fatbin") as f:
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={f.name}", path, "/dev/null"],
                       check=True)
        blob = open(f.name, "rb").read()
    pos = 0
    while True:
        pos = blob.find(b"__CLANG_OFFLOAD_BUNDLE__", pos)
        if pos < 0:
            return
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, q)
            triple = blob[q + 24:q + 24 + tl].decode()
            q += 24 + tl
            if "gfx950" in triple:
                yield blob[pos + off:pos + off + size]
        pos += 1


def main():
    path, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    for co in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
        entries, cur = [], None
        for line in notes.splitlines():
            if line.strip().startswith("- .agpr_count:"):
                cur = {"agpr": line.split(":")[1].strip()}
                entries.append(cur)
                continue
            m = re.match(r"\s+\.(\w+):\s+(.*)", line)
            if m and cur is not None and m.group(1) in ("name", "group_segment_fixed_size", "private_segment_fixed_size",
                                                        "vgpr_count", "vgpr_spill_count", "sgpr_count"):
                cur.setdefault(m.group(1), m.group(2))
        for e in entries:
            v = e.get("name", "")
            if sub in v:
                dem = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
                print(f"vgpr {e.get('vgpr_count')} agpr {e.get('agpr')} spill {e.get('vgpr_spill_count')} "
                      f"scratch {e.get('private_segment_fixed_size')} lds {e.get('group_segment_fixed_size')}  {dem}")

if __name__ == "__main__":
    main()
