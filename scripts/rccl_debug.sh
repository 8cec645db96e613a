#!/bin/bash
# Diagnose RCCL bootstrap on the GPU box (torch ProcessGroupNCCL vs direct RCCL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export AHV_SKIP_AUTOBUILD=1
timeout -k 10 120 env MASTER_ADDR=127.0.0.1 MASTER_PORT=29511 RANK=0 WORLD_SIZE=1 python -c "
import torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda',0))
x=torch.ones(4, device='cuda'); dist.all_reduce(x); torch.cuda.synchronize(); print('torch nccl ok', x.tolist())
dist.destroy_process_group()
" > gpurun_out/rccl_torch.log 2>&1; echo "torch rc=$?"
timeout -k 10 120 env NCCL_DEBUG=INFO python -c "
import torch
torch.zeros(1, device='cuda'); torch.cuda.synchronize()
from agent_hypervisor_amd._native import C
print('version', C.rccl_version())
print('uid', len(C.rccl_unique_id()))
" > gpurun_out/rccl_direct.log 2>&1; echo "direct rc=$?"
tail -30 gpurun_out/rccl_torch.log; tail -40 gpurun_out/rccl_direct.log
