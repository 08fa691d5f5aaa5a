"""Frame-per-GPU sharding with the one real exchange of the path: the luminance-histogram all-reduce.

SURVEY.md §8e: frames are independent units; rank r renders camera r with its own TAA history. Global
auto-exposure is the only cross-GPU dependency. After GenerateLuminanceHistogram each rank holds 256 u32
bins, RCCL all-reduces them (1 KiB over xGMI, backend "nccl"), and every rank then resolves the same
exposure with total_pixels = N*W*H and a 64-bit weighted sum (the reference's u32 sum would overflow
for 8 frames). The helpers are device-agnostic so the N>1 logic is testable with gloo on CPU.
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

SPONZA_CAMERA = ((-14.0, 2.2, 0.3), (0.0, -0.42, 0.0))
# config C4: above the fBm terrain looking down the diagonal, f_sky ~= 0.5 at 16:9
TERRAIN_CAMERA = ((20.0, 34.0, 20.0), (0.785, 0.6, 0.0))


def env() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


# exchange even without peers (init(force_exchange=True)): a world-size-1 group still runs the real collective, so
# the PRE -> all-reduce -> POST path (RCCL on the AutoExposure bins) is exercised on a 1-GPU box
_FORCE_EXCHANGE = False


def init(device: Optional[torch.device] = None, backend: str = "nccl", force_exchange: bool = False) -> None:
    """Join the process group (torch.distributed.run environment). Without peers nothing is initialised unless
    `force_exchange`: then a world-size-1 group is created and every frame takes the exchange path."""
    global _FORCE_EXCHANGE
    _, world, _ = env()
    _FORCE_EXCHANGE = bool(force_exchange)
    if (world > 1 or force_exchange) and not dist.is_initialized():
        if world == 1:   # no launcher: a one-rank rendezvous on the loopback address
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("LOCAL_RANK", "0")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket
                s = socket.socket()
                s.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s.getsockname()[1])
                s.close()
        if backend == "nccl":
            dist.init_process_group(backend, device_id=device)
        else:
            dist.init_process_group(backend)


def exchange_active(group=None) -> bool:
    """True when frames take PRE -> histogram all-reduce -> POST (peers, or a forced world-size-1 group)."""
    return dist.is_initialized() and (dist.get_world_size(group) > 1 or _FORCE_EXCHANGE)


def camera_for_rank(rank: int):
    """Rank 0: the canonical Sponza-proxy view; others: seeded poses along the nave (seed 0xC5 + rank)."""
    if rank == 0:
        return SPONZA_CAMERA
    rng = np.random.default_rng(0xC5 + rank)
    pos = (float(rng.uniform(-15.0, 12.0)), float(rng.uniform(1.5, 4.0)), float(rng.uniform(-2.5, 2.5)))
    rot = (float(rng.choice([0.0, math.pi])) + float(rng.uniform(-0.3, 0.3)), float(rng.uniform(-0.6, -0.2)), 0.0)
    return pos, rot


def terrain_camera_for_rank(rank: int):
    """Rank 0: the canonical C4 view; others: seeded headings and heights over the terrain (seed 0xC4 + rank)."""
    if rank == 0:
        return TERRAIN_CAMERA
    rng = np.random.default_rng(0xC4 + rank)
    pos = (float(rng.uniform(15.0, 30.0)), float(rng.uniform(32.0, 40.0)), float(rng.uniform(15.0, 30.0)))
    return pos, (0.785 + float(rng.uniform(-0.5, 0.5)), float(rng.uniform(0.5, 0.7)), 0.0)


def exposure_pixels(world: int, width: int, height: int) -> Tuple[int, bool]:
    """(total_pixels, wide_accumulator) for the resolve after the histogram exchange."""
    return world * width * height, world > 1


def exchange_histogram(bins: torch.Tensor, group=None) -> None:
    """Sum the per-rank 256-bin histograms in place (u32 bins viewed as int32: two's-complement wrap)."""
    if exchange_active(group):
        dist.all_reduce(bins, op=dist.ReduceOp.SUM, group=group)


def max_over_ranks(x: float, device=None) -> float:
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def render_frame(renderer, g, bins: torch.Tensor, group=None, exchange_events=None) -> None:
    """One frame of the sharded path: PRE phase, histogram exchange, POST phase (all on the frame stream).
    Without peers the frame is one call (the resolve then folds the fused pass's partial histograms).
    `exchange_events` = (start, end) CUDA events recorded on the current stream around the exchange."""
    from . import PHASE_ALL, PHASE_POST_EXPOSURE, PHASE_PRE_EXPOSURE
    if not exchange_active(group):
        renderer.execute(g, PHASE_ALL)
        return
    renderer.execute(g, PHASE_PRE_EXPOSURE)
    if exchange_events is not None:
        exchange_events[0].record()
    exchange_histogram(bins, group)
    if exchange_events is not None:
        exchange_events[1].record()
    renderer.execute(g, PHASE_POST_EXPOSURE)


def rank_inventory(device) -> dict:
    """What this rank runs on: the device the collective backend sees (index, name, PCI bus id)."""
    props = torch.cuda.get_device_properties(device)
    bus = getattr(props, "pci_bus_id", None)
    return {"device_index": device.index, "name": props.name,
            "pci": (f"{getattr(props, 'pci_domain_id', 0):04x}:{bus:02x}:{getattr(props, 'pci_device_id', 0):02x}"
                    if bus is not None else None)}


def gather_objects(obj):
    """all_gather_object over the world (a list of one object without peers)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
