# per-kernel VGPR / SGPR / scratch / LDS of a built libnimble_amd.so (the
# gfx950 code object's metadata): tools/kernel_resources.sh [lib]
set -e
LIB=$(realpath ${1:-nimblephysics_amd/libnimble_amd.so})
D=$(mktemp -d)
cd $D
objcopy --dump-section .hip_fatbin=fb.bin $LIB
T=$(/opt/rocm/llvm/bin/clang-offload-bundler --list --type=o --input=fb.bin | grep gfx950 | head -1)
/opt/rocm/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=$T --input=fb.bin --output=co.o
/opt/rocm/llvm/bin/llvm-readelf --notes co.o > notes.txt
python3 - <<'PY'
import re
t = open("notes.txt").read()
for blk in t.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or not name.group(1).startswith("nimble_"):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    print(f"{name.group(1):34s} vgpr {g('vgpr_count'):>4s} sgpr {g('sgpr_count'):>4s} scratch {g('private_segment_fixed_size'):>6s} "
          f"vgpr_spill {g('vgpr_spill_count'):>4s} lds {g('group_segment_fixed_size')}")
PY
rm -rf $D
