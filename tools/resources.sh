#!/bin/bash
# Per-kernel VGPRs / scratch of every fused spec (compiler view, no GPU).
cd /tmp
for k in 0 1 2 3 4 5; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I /root/repo/include -DTDBG_PART=$k -DTDBG_NPART=6 \
    -c /root/repo/tiledb_amd/csrc/tdbg_fast.hip -o /tmp/tdbg_res_p$k.o -Rpass-analysis=kernel-resource-usage 2>&1 |
    grep -E "Function Name|VGPRs:|ScratchSize" | sed 's/.*remark: //; s/ \[-Rpass.*//; s/.*kernel-resource-usage\]//' |
    sed 's/^.*\(Function Name\|VGPRs\|ScratchSize\)/\1/' | paste - - - | sed 's/Function Name: _ZN4tdbg21unfilter_fused_kernel//'
done
