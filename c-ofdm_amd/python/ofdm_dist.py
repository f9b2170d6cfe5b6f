"""ofdm_dist — frame sharding and the one end-of-job reduction.

Frames are independent (own pilots, own symbol-0 reference, own sync), so a
batch shards as contiguous frame ranges, remainder to the low ranks, with no
data-path collective. The only collective is a SUM all-reduce of the
{bit_errors, bits, samples, frames} counters plus a MAX of the elapsed time
(RCCL over xGMI on MI355X, gloo in the CPU tests)."""
from __future__ import annotations

import os


def shard(n_units: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [begin, begin+count) of n_units for `rank`; low ranks take the remainder."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, rem = divmod(n_units, world)
    count = base + (1 if rank < rem else 0)
    begin = rank * base + min(rank, rem)
    return begin, count


def env_world() -> tuple[int, int, int]:
    """(world, rank, local_rank) from torch.distributed.run's environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def reduce_counters(counters, dist=None):
    """SUM all-reduce of an int64 tensor [bit_errors, bits, samples, frames]
    (in place; a GPU tensor under gloo is reduced through a host copy)."""
    if dist is not None and dist.is_initialized():
        if dist.get_backend() == "gloo" and counters.is_cuda:
            h = counters.cpu()
            dist.all_reduce(h)
            counters.copy_(h)
        else:
            dist.all_reduce(counters)
    return counters


def max_over_ranks(value: float, device, dist=None) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=collective_device(dist, device))
    if dist is not None and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(nprocs: int, script: str, argv: list[str], env: dict | None = None,
                 capture: bool = False):
    """Start `nprocs` ranks of `script` on this node with torch.distributed.run
    (one process per GPU; rendezvous on 127.0.0.1) and wait for them. The
    caller must not have touched the GPU: the ranks are child processes, the
    caller only waits. Returns the launcher's exit code, or (code, stdout) with
    capture=True (rank 0's JSON line is on stdout)."""
    import subprocess
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nprocs}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", script, *argv]
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("OMP_NUM_THREADS", "1")
    if capture:
        r = subprocess.run(cmd, env=e, stdout=subprocess.PIPE, text=True)
        return r.returncode, r.stdout
    return subprocess.call(cmd, env=e)


def needs_launch(gpus: int) -> bool:
    """True when `--gpus N` (N > 1) was asked for and this process is not
    already one rank of a launched job (no WORLD_SIZE in the environment)."""
    return gpus > 1 and "WORLD_SIZE" not in os.environ


def init(backend: str, local_rank: int, use_gpu: bool = True):
    """Bind this rank to its device and join the process group (world > 1).
    nccl = RCCL over xGMI, one GPU per rank (needs local_rank < device count);
    gloo = CPU collectives, several ranks may share a GPU (test rehearsal).
    Returns (torch.distributed or None, device)."""
    import torch
    world, _, _ = env_world()
    dev = torch.device("cpu")
    if use_gpu:
        ndev = torch.cuda.device_count()
        if backend == "nccl" and world > 1 and local_rank >= ndev:
            raise RuntimeError(f"rank {local_rank} of {world} needs its own GPU (nccl/RCCL) but {ndev} are visible; "
                               "use --backend gloo to rehearse several ranks on one GPU")
        dev = torch.device("cuda", local_rank % max(ndev, 1))
        torch.cuda.set_device(dev)
    # a launched job (WORLD_SIZE set) joins the group even at one rank, so the
    # RCCL reduction path runs under `torch.distributed.run --nproc-per-node 1`
    if world == 1 and "WORLD_SIZE" not in os.environ:
        return None, dev
    import torch.distributed as dist
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    return dist, dev


def collective_device(dist, device):
    """Where the reduction tensors live: the GPU for RCCL, the host for gloo."""
    import torch
    if dist is not None and dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return device
