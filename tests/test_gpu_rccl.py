"""The RCCL path on the GPU box (one GPU): a world-1 process group over the `nccl` backend (RCCL),
started the way bench.py --gpus N starts its ranks (stablekeypoints_amd.launch.spawn_ranks →
torch.distributed.run), with bench.py's init call (device_id bound), then the step's collectives:
the flat fp32 SUM all-reduce of TokenOptimizer.optimizer_step, the fp64 MAX all-reduce of the
timed region and a barrier.  The N > 1 RCCL runs need a multi-GPU node (the driver's SCALE runs);
this checks the backend, the launcher and the calls on the box's own stack."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, torch, torch.distributed as dist
local = int(os.environ["LOCAL_RANK"])
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
assert dist.get_backend() == "nccl" and dist.get_world_size() == int(os.environ["WORLD_SIZE"])
flat = torch.arange(500 * 768 + 3, device="cuda", dtype=torch.float32)
ref = flat.clone() * dist.get_world_size()
dist.all_reduce(flat, op=dist.ReduceOp.SUM)
assert torch.equal(flat, ref)
t = torch.tensor([1.5 + dist.get_rank()], device="cuda", dtype=torch.float64)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert float(t.item()) == 1.5 + dist.get_world_size() - 1
dist.barrier()
torch.cuda.synchronize()
dist.destroy_process_group()
print("rccl ok", flush=True)
'''


@pytest.mark.gpu
def test_rccl_world1_through_the_launcher(tmp_path):
    sys.path.insert(0, REPO)
    from stablekeypoints_amd.launch import spawn_ranks
    script = tmp_path / "rccl_worker.py"
    script.write_text(WORKER)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = spawn_ranks(1, [str(script)], [], env=env)
    assert rc == 0
