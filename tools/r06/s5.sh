#!/bin/bash
# round 6, GPU session 5: (a) the GPU's state over the first seconds of load -- the same per-tile and LDS-DMA commands
# without and with a 3 s pre-warm, five rounds, every measurement's clocks / power; (b) rocprofv3 kernel trace of the
# LDS-DMA form at N = 32 (A/B variant 1536) for the per-launch durations and the gaps between launches
set -u
O=gpurun_out/r06_s5
mkdir -p $O
export TMPDIR=/tmp
L=nvflare_amd/lib/ab/dma_ab.so
python -c "
import json, amdsmi
amdsmi.amdsmi_init()
h = amdsmi.amdsmi_get_processor_handles()[0]
m = amdsmi.amdsmi_get_gpu_metrics_info(h)
print(json.dumps({k: (v if isinstance(v, (int, float, str)) else str(v)) for k, v in m.items()}))
for t in ('SYS', 'MEM', 'DF', 'SOC', 'FCLK'):
    try:
        print(t, json.dumps(amdsmi.amdsmi_get_clk_freq(h, getattr(amdsmi.AmdSmiClkType, t)), default=str))
    except Exception as e:
        print(t, 'n/a', e)
" > $O/amdsmi_dump.txt 2>&1
NVFLARE_AMD_FEDAVG_LIB=$L timeout -k 10 400 python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 4,1536 --epilogues adam --rounds 5 --sqrt torch_cpu_amd > $O/ab_k2_cold.jsonl 2> $O/ab_k2_cold.err &&
NVFLARE_AMD_FEDAVG_LIB=$L timeout -k 10 400 python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 4,1536 --epilogues adam --rounds 5 --prewarm-s 3 --sqrt torch_cpu_amd > $O/ab_k2_warm.jsonl 2> $O/ab_k2_warm.err &&
NVFLARE_AMD_FEDAVG_LIB=$L timeout -k 10 400 python -u tools/ab_variants.py --clients 3 --params 1e9 --variants 4,1536 --epilogues adam --rounds 5 --prewarm-s 3 --sqrt torch_cpu_amd > $O/ab_k3_warm.jsonl 2> $O/ab_k3_warm.err &&
NVFLARE_AMD_FEDAVG_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp_n32 -o n32 -- python3 tools/ab_variants.py --clients 2 --params 1e9 --variants 1536 --epilogues adam --rounds 2 --sqrt torch_cpu_amd > $O/rp_n32.jsonl 2> $O/rp_n32.err
echo "rc=$?"
