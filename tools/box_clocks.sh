#!/bin/bash
# GPU box, diagnostics only: does the batch kernel's placement level follow the box's
# clocks?  Records the SMI view of the box (clocks, memory partition, firmware), then the C3 batch
# bench, then the clocks again (under load the DPM states have settled).  Output under
# gpurun_out/box/<tag>/.
tag=${1:-box}
o=gpurun_out/box/$tag; mkdir -p $o
timeout -k 5 60 rocm-smi --showclocks > $o/clocks_before.txt 2>&1
timeout -k 5 60 rocm-smi --showmemvendor --showproductname --showvbios --showmeminfo vram --showpids > $o/product.txt 2>&1
timeout -k 5 60 amd-smi static --partition --clock > $o/amdsmi_static.txt 2>&1
timeout -k 5 60 amd-smi metric --clock > $o/amdsmi_clock_before.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --no-cpu > $o/bench_c3.log 2>&1 || exit 1
timeout -k 5 60 amd-smi metric --clock > $o/amdsmi_clock_after.txt 2>&1
timeout -k 5 60 rocm-smi --showmeminfo vram --showpids > $o/mem_after.txt 2>&1
timeout -k 5 60 python -c "import torch; f, t = torch.cuda.mem_get_info(0); print('free', f, 'total', t)" > $o/mem_get_info.txt 2>&1
tail -1 $o/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['roofline']['frac'], d['roofline']['kernel_ms_avg'])"
