"""One rank of tests/test_gpu_parity.py::test_row_parallel_rccl_two_ranks:
RowParallelLinear (HIP NT GEMM) + dist.all_reduce on the "nccl" (RCCL)
backend over xGMI; rank 0 checks the sum against the full product in f64.
Exit code 0 = pass."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "physics-llm-inference_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import linear as olin  # noqa: E402
from oracle.numerics import seeded_normal  # noqa: E402


def main():
    rank, world = int(sys.argv[1]), int(sys.argv[2])
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", device_id=torch.device("cuda", rank))
    from ch09 import RowParallelLinear
    M, K, N = 512, 2048, 1024
    x = seeded_normal((M, K), 5, "bf16")
    w = seeded_normal((N, K), 6, "bf16")
    ks = K // world
    sl = slice(rank * ks, (rank + 1) * ks)
    layer = RowParallelLinear(K, N, world_size=world, rank=rank).cuda().to(torch.bfloat16)
    layer.weight.data.copy_(torch.from_numpy(np.ascontiguousarray(w[:, sl])).cuda().to(torch.bfloat16))
    with torch.no_grad():
        y = layer(torch.from_numpy(np.ascontiguousarray(x[:, sl])).cuda().to(torch.bfloat16)).float()
    mag = y.abs().clone()
    dist.all_reduce(y)
    dist.all_reduce(mag)
    ok = True
    if rank == 0:
        ref = olin.linear(x, w)
        err = np.abs(y.cpu().numpy().astype(np.float64) - ref)
        ok = bool(np.all(err <= 1e-2 * (mag.cpu().numpy() + 1.0)))
        print("rccl row-parallel max err", err.max(), "ok", ok, flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
