"""One rank of tests/test_gpu_rccl.py: the HIP library and RCCL ("nccl"
backend) in one process.  Row-parallel forward of ch09 (reference
ch09/tensor_parallel.py:43-68) on a process group passed explicitly:

1. RowParallelLinear (bf16 partials, pli_gemm NT) + dist.all_reduce;
2. row_parallel_forward_overlapped(chunks=4): each chunk's async all-reduce
   on RCCL's stream after that chunk's pli_gemm on the current stream;
3. the fp32-partial path (reduce_dtype=torch.float32, pli_gemm_f32out) in
   both forms.

At world size 1 the all-reduce is the identity, so every result must be
bitwise equal to the same GEMMs run without the group (which also proves the
collective ran after the GEMM that fills its buffer); at world size 2 the
chunked and plain forms must agree within one output rounding (not bitwise:
RCCL may pick a different reduction schedule for a 128-row chunk than for
the whole buffer, and the small-M GEMM a different route), and every form
must match a float64 product within its rounding bound.  Prints one JSON
line; exit code 0 = pass.  argv: rank world.

UNVERIFIED ON HARDWARE: the world-size-2 leg has never run -- the GPU pool of
every round so far had one GPU per box, so tests/test_gpu_rccl.py skips it;
only the world-size-1 leg (RCCL + the HIP library in one process) has run."""
import json
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
    dev = rank % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    import pli_hip
    from ch09 import RowParallelLinear, row_parallel_forward_overlapped
    group = dist.group.WORLD
    M, K, N = 512, 2048, 1024
    x = seeded_normal((M, K), 5, "bf16")
    w = seeded_normal((N, K), 6, "bf16")
    ks = K // world
    sl = slice(rank * ks, (rank + 1) * ks)
    xs = torch.from_numpy(np.ascontiguousarray(x[:, sl])).cuda().to(torch.bfloat16)
    ws = torch.from_numpy(np.ascontiguousarray(w[:, sl])).cuda().to(torch.bfloat16)
    bounds = [M * i // 4 for i in range(5)]
    res = {"rank": rank, "world": world, "backend": dist.get_backend()}
    ok = True
    with torch.no_grad():
        layer = RowParallelLinear(K, N, world_size=world, rank=rank, group=group).cuda().to(torch.bfloat16)
        layer.weight.data.copy_(ws)
        l32 = RowParallelLinear(K, N, world_size=world, rank=rank, group=group,
                                reduce_dtype=torch.float32).cuda().to(torch.bfloat16)
        l32.weight.data.copy_(ws)
        y = layer(xs)
        y2 = row_parallel_forward_overlapped(xs, ws, chunks=4, group=group, world_size=world)
        y3 = l32(xs)
        y4 = row_parallel_forward_overlapped(xs, ws, chunks=4, group=group, world_size=world,
                                             reduce_dtype=torch.float32)
        # the same GEMMs without any collective
        p = pli_hip.gemm(xs, ws, trans_b=True)
        pc = torch.cat([pli_hip.gemm(xs[lo:hi], ws, trans_b=True) for lo, hi in zip(bounds, bounds[1:])])
        p32 = pli_hip.gemm_f32out(xs, ws)
        pc32 = torch.cat([pli_hip.gemm_f32out(xs[lo:hi], ws) for lo, hi in zip(bounds, bounds[1:])])
        mag = p.float().abs()
        torch.cuda.synchronize()
    if world == 1:
        checks = {"layer_eq_gemm": torch.equal(y, p), "overlapped_eq_chunked_gemm": torch.equal(y2, pc),
                  "f32_layer_eq_gemm_f32out": torch.equal(y3, p32.to(torch.bfloat16)),
                  "f32_overlapped_eq_chunked": torch.equal(y4, pc32.to(torch.bfloat16))}
    else:
        pcs = pc_sum(pc)  # every rank calls the collective

        def one_rounding(a, b):  # |a - b| within a bf16 rounding of either (+ fp32 order effects)
            a, b = a.float(), b.float()
            return bool(((a - b).abs() <= 2.0 ** -7 * torch.maximum(a.abs(), b.abs()) + 1e-3).all())
        checks = {"overlapped_vs_chunked_allreduce": one_rounding(y2, pcs),
                  "f32_overlapped_vs_layer": one_rounding(y4, y3)}
        res["f32_overlapped_vs_layer_max_diff"] = (y4.float() - y3.float()).abs().max().item()
    dist.all_reduce(mag)
    ref = olin.linear(x, w)
    bound = 1e-2 * (mag.cpu().numpy() + 1.0)
    for name, val, tight in (("layer", y, False), ("overlapped", y2, False), ("f32_layer", y3, True),
                             ("f32_overlapped", y4, True)):
        err = np.abs(val.float().cpu().numpy().astype(np.float64) - ref)
        # fp32 partials: one bf16 rounding of the sum (2^-8 relative) + fp32 accumulation
        lim = (2.0 ** -8 * np.abs(ref) + 1e-4 * (mag.cpu().numpy() + 1.0)) if tight else bound
        checks[f"{name}_vs_f64"] = bool(np.all(err <= lim))
        res[f"{name}_max_err"] = float(err.max())
    res["checks"] = {k: bool(v) for k, v in checks.items()}
    ok = all(res["checks"].values())
    res["ok"] = ok
    print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


def pc_sum(pc):
    out = pc.clone()
    dist.all_reduce(out)
    return out


if __name__ == "__main__":
    main()
