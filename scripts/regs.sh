#!/bin/bash
# register usage of the kernels in kcc_kernels.hip (device-only asm)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I/root/repo/include -I/root/repo/kubernetesclustercapacity_amd/csrc --cuda-device-only -S -o /tmp/k.s /root/repo/kubernetesclustercapacity_amd/csrc/${1:-kcc_kernels.hip} "${@:2}" 2>&1 | grep -v "hip-link"
python3 - <<'PY'
import re
s=open('/tmp/k.s').read()
for blk in s.split('- .agpr_count')[1:]:
    name=re.search(r'\.name:\s+(\S+)',blk).group(1)
    g=lambda k: re.search(r'\.'+k+r':\s+(\d+)',blk).group(1)
    print(f"{name[:58]:58s} sgpr={g('sgpr_count')} vgpr={g('vgpr_count')} lds={g('group_segment_fixed_size')} scratch={g('private_segment_fixed_size')}")
PY
