set -e
cd /root/repo
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -o nimblephysics_amd/libnimble_amd.so nimblephysics_amd/csrc/timestep.hip nimblephysics_amd/csrc/capi.cpp nimblephysics_amd/csrc/world_api.cpp nimblephysics_amd/csrc/loaders.cpp 2>&1 | grep -E "error|warning: v" -A3 || true
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -DNIMBLE_STAGE_TIMING -o dbg/libnimble_dbg.so nimblephysics_amd/csrc/timestep.hip nimblephysics_amd/csrc/capi.cpp nimblephysics_amd/csrc/world_api.cpp nimblephysics_amd/csrc/loaders.cpp 2>&1 | grep error -A3 || true
