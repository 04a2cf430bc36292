#!/bin/bash
# Round 4: PCIe copy engines (SDMA vs copy kernels, both directions at once), and which HIP runtime
# a torch process loads.
set -u
mkdir -p gpurun_out
timeout -k 10 200 tools/pcie_pattern 1024 > gpurun_out/r04e_pcie_engines.txt 2>&1 || { echo pp FAILED; tail gpurun_out/r04e_pcie_engines.txt; exit 1; }
grep engines gpurun_out/r04e_pcie_engines.txt
timeout -k 10 120 python -c "
import torch, ctypes
torch.zeros(1, device='cuda')
ctypes.CDLL('arpc_amd/lib/libsymphony_hip.so')
print(sorted({l.split()[-1] for l in open('/proc/self/maps') if 'amdhip' in l or 'hsa-runtime' in l}))
" > gpurun_out/r04e_libs.txt 2>&1
cat gpurun_out/r04e_libs.txt
echo r04e ok
