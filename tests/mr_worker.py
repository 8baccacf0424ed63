"""One rank of the multi-process parity test (tests/test_gpu_parity.py).

usage: mr_worker.py <snpfile> <out> [options...]  (RANK/WORLD_SIZE/MASTER_* in env)
Exchange over torch.distributed gloo (CPU tensors) so that two ranks can share
one GPU, or (FSCL_MR_SHM=<name>) the library's own shared-memory exchange.
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import fscl_amd  # noqa: E402
from test_gpu_parity import _kw  # noqa: E402


def main() -> int:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce(arr: np.ndarray) -> None:
        t = torch.from_numpy(arr)  # shares memory with the C buffer
        dist.all_reduce(t, op=dist.ReduceOp.SUM)

    if os.environ.get("FSCL_MR_SHM"):  # the library's own shared-memory exchange
        fscl_amd.set_ranks_shm(rank, world, os.environ["FSCL_MR_SHM"])
    else:
        fscl_amd.set_ranks(rank, world, allreduce)
    snp, out, opts = sys.argv[1], sys.argv[2], sys.argv[3:]
    fscl_amd.run(snp, out, **_kw(opts))
    st = fscl_amd.get_stats()
    dist.barrier()
    print(f"rank {rank}: gp_evals {st['gp_evals']} spec_threads {st['spec_threads']} negj {st['negj']} "
          f"perm_leader {st['perm_leader']} plan_mode {st['plan_mode']} plan_fallback {st['plan_fallback']}",
          file=sys.stderr)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
