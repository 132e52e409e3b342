#!/bin/bash
# VGPR / spill report of the tile sweep kernel instantiations (compile only)
cd "$(dirname "$0")/../improving-performances-of-mcmc-for-nearest-neighbor-gaussian-process-models-with-full-data-augmentat_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-pass-failed -Wno-unused-value -Wno-unused-result -c tiles.hip -o /tmp/tile_regs.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep -A12 "Name: _ZN4nngp18sweep_tiles_kernel" | grep -E "Function Name|VGPRs:|VGPRs Spill|ScratchSize" \
 | sed -e 's/.*remark: //' -e 's/ \[-Rpass.*//' | paste - - - - | sed 's/_ZN4nngp18sweep_tiles_kernelIL//'
