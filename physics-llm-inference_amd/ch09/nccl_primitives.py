"""Collective cost models -- mirror of ``ch09/nccl_primitives.py`` plus the
MI355X xGMI bounds used to judge the measured RCCL all-reduce.

The four reference models are kept with identical results, including the
reference's unit convention: ``bandwidth_gbps`` is divided by 8 (treated as
Gbit/s) in ``simulate_all_reduce``/``simulate_all_gather``/
``compute_ring_all_reduce_time`` (``:25,52,80``).  ``xgmi_all_reduce_bounds``
is new and uses GB/s (bytes) throughout.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class AllReduceConfig:
    world_size: int = 8
    data_size_mb: float = 1.0
    bandwidth_gbps: float = 600.0
    latency_us: float = 5.0


@dataclass
class AllGatherConfig:
    world_size: int = 8
    data_size_per_gpu_mb: float = 1.0
    bandwidth_gbps: float = 600.0
    latency_us: float = 5.0


def _bytes_per_us(gbps: float) -> float:
    return gbps * 1e9 / 8 / 1e6  # reference convention (Gbit/s)


def simulate_all_reduce(config: AllReduceConfig) -> dict:
    """Ring all-reduce: 2 (n-1)/n of the payload crosses each link."""
    data = config.data_size_mb * 1024 * 1024
    moved = 2 * data * (config.world_size - 1) / config.world_size
    transfer = moved / _bytes_per_us(config.bandwidth_gbps)
    total = config.latency_us + transfer
    eff = data / (total * 1e-6) / 1e9
    return {"data_size_mb": config.data_size_mb, "world_size": config.world_size,
            "transfer_bytes": moved, "latency_us": config.latency_us,
            "transfer_time_us": transfer, "total_time_us": total,
            "effective_bandwidth_gbps": eff,
            "bandwidth_efficiency": eff / config.bandwidth_gbps}


def simulate_all_gather(config: AllGatherConfig) -> dict:
    """Each rank receives the other n-1 shards."""
    per = config.data_size_per_gpu_mb * 1024 * 1024
    total_bytes = per * config.world_size
    transfer = per * (config.world_size - 1) / _bytes_per_us(config.bandwidth_gbps)
    total = config.latency_us + transfer
    return {"data_per_gpu_mb": config.data_size_per_gpu_mb,
            "total_data_mb": total_bytes / 1024 / 1024, "world_size": config.world_size,
            "transfer_time_us": transfer, "total_time_us": total,
            "effective_bandwidth_gbps": total_bytes / (total * 1e-6) / 1e9}


def compute_ring_all_reduce_time(data_size_bytes: int, world_size: int,
                                 bandwidth_gbps: float = 600.0, latency_us: float = 5.0) -> float:
    """2 (n-1) ring steps, each moving one 1/n chunk plus a fixed latency."""
    step = latency_us + (data_size_bytes / world_size) / _bytes_per_us(bandwidth_gbps)
    return 2 * (world_size - 1) * step


def compute_communication_overlap_potential(compute_time_us: float, comm_time_us: float) -> dict:
    seq = compute_time_us + comm_time_us
    ovl = max(compute_time_us, comm_time_us)
    return {"compute_time_us": compute_time_us, "comm_time_us": comm_time_us,
            "sequential_time_us": seq, "overlapped_time_us": ovl,
            "potential_speedup": seq / ovl,
            "overlap_ratio": min(compute_time_us, comm_time_us) / ovl,
            "bottleneck": "compute" if compute_time_us >= comm_time_us else "communication"}


def xgmi_all_reduce_bounds(payload_bytes: float, world_size: int,
                           link_gbps: float = 153.0, links: int = 7) -> dict:
    """Lower bounds (us) for an all-reduce of ``payload_bytes`` per rank on
    MI355X xGMI: point-to-point links, ``links`` per GPU at ``link_gbps`` GB/s.

    single ring  : 2 (n-1)/n * S over ONE outbound link per GPU;
    full mesh    : reduce-scatter + all-gather spread over the n-1 direct links,
                   2 (n-1)/n * S / ((n-1) * link) = 2 S / (n * link).
    busbw convention (nccl-tests): busbw = S / t * 2 (n-1) / n.
    """
    n = world_size
    if n <= 1:
        return {"ring_us": 0.0, "mesh_us": 0.0}
    ring = 2 * (n - 1) / n * payload_bytes / (link_gbps * 1e3)
    mesh = 2 * (n - 1) / n * payload_bytes / (min(n - 1, links) * link_gbps * 1e3)
    return {"ring_us": ring, "mesh_us": mesh,
            "bus_factor": 2 * (n - 1) / n}


def explain_nccl() -> str:
    """The reference's collective-communication primer
    (ch09/nccl_primitives.py:110-147), written for this build: on ROCm the
    "nccl" backend of torch.distributed is RCCL, and MI355X GPUs talk over
    point-to-point xGMI links instead of a switch."""
    return (
        "\nRCCL (the ROCm collectives behind torch.distributed's \"nccl\" backend)\n\n"
        "Collectives a tensor-parallel / expert-parallel model uses:\n"
        "  all-reduce      every rank ends with the sum of all ranks' buffers\n"
        "                  (the row-parallel layer's partial products); ring cost\n"
        "                  2 (N-1)/N x bytes per rank on the slowest link\n"
        "  all-gather      every rank ends with every rank's shard, (N-1)/N x the\n"
        "                  gathered bytes per rank\n"
        "  reduce-scatter  the sum, with rank r keeping its 1/N slice (half an\n"
        "                  all-reduce)\n"
        "  all-to-all      rank r sends a different slice to every rank (MoE token\n"
        "                  routing)\n\n"
        "Ring all-reduce: the buffer is cut into N chunks; N-1 reduce steps pass\n"
        "partial sums around the ring, N-1 gather steps pass the finished chunks.\n\n"
        "MI355X fabric: each GPU has 7 xGMI links (~153 GB/s each) to the other 7\n"
        "GPUs of the node -- a full mesh, not a switch -- so a single ring runs at\n"
        "one link's rate, while a collective that uses all links at once is bounded\n"
        "by 2 x bytes / (N x 153 GB/s) (xgmi_all_reduce_bounds).  Tensor-parallel\n"
        "layers therefore chunk the all-reduce and overlap it with the next GEMM\n"
        "(tensor_parallel.row_parallel_forward_overlapped).\n"
    )


if __name__ == "__main__":
    # the chapter's demo (ch09/nccl_primitives.py:149-181): ring all-reduce
    # model at the reference's 600 GB/s link, then compute / comm overlap
    print(explain_nccl())
    print("\n" + "=" * 60 + "\nAll-Reduce Simulation\n" + "-" * 60)
    for n in (2, 4, 8):
        r = simulate_all_reduce(AllReduceConfig(world_size=n, data_size_mb=100.0, bandwidth_gbps=600.0))
        print(f"\nWorld size: {n}\n  Data size: {r['data_size_mb']:.1f} MB\n  Total time: {r['total_time_us']:.1f} us\n"
              f"  Effective bandwidth: {r['effective_bandwidth_gbps']:.1f} GB/s\n"
              f"  Efficiency: {r['bandwidth_efficiency']:.1%}")
        b = xgmi_all_reduce_bounds(100.0 * 2**20, n)
        print(f"  MI355X xGMI bounds: {b}")
    print("\n" + "=" * 60 + "\nCommunication-Compute Overlap Analysis\n" + "-" * 60)
    for compute_us in (100, 500, 1000):
        o = compute_communication_overlap_potential(compute_us, 200)
        print(f"\nCompute: {compute_us} us, Comm: 200 us\n  Sequential: {o['sequential_time_us']:.0f} us\n"
              f"  Overlapped: {o['overlapped_time_us']:.0f} us\n  Speedup: {o['potential_speedup']:.2f}x\n"
              f"  Bottleneck: {o['bottleneck']}")
