#!/bin/bash
# Register / scratch usage of the van der Pol solve kernel (its pair translation unit).
cd /tmp && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC "$@" -I/root/repo/include \
  -I/root/repo/nlp-filter_amd/csrc -c /root/repo/nlp-filter_amd/csrc/pair_vdp.hip -o /tmp/resusage.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -A12 "Function Name: _ZN3mhe4k_gnINS_12DynVanDerPol.*ELi0ELb0E" | grep -E "Function Name|VGPRs:|AGPRs|Spill|ScratchSize|Occupancy|LDS"
