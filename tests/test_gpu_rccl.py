"""The RCCL branch of the N-GPU path on hardware (one GPU, world size 1): an
`nccl` process group (RCCL on ROCm) carries TileGather's framebuffer gather
(sptamd/distributed.py, the path's only exchange step) and the
bench's max-over-ranks all-reduce on CUDA tensors (bench.py timed_loop), so the
code the 8-GPU run takes has executed on an MI355X.  The gathered image must
equal the rendered tile bit for bit and the oracle's image."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

import oracle as O
import sptamd
from sptamd import scenes
from sptamd.distributed import TileGather

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_gather_and_allreduce_world1():
    assert not dist.is_initialized()
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        mesh = scenes.mitsuba_synth(detail=0.1)
        s = sptamd.Scene()
        s.add_arrays(mesh)
        s.commit(0)
        W, H, spp, D = 96, 64, 4, 4
        tg = TileGather(H, W, 0, 1, 8, dev)
        assert tg.collective and tg.gather_list is not None
        for k in (0, 1):  # both film buffers, as bench.py alternates them
            film = tg.tile_view(k)
            s.render(sptamd.make_params(W, H, spp, D, tile_index=0, tile_count=1, rows_per_group=8), film=film)
            img = tg.gather(k)  # dist.gather over RCCL
            torch.cuda.synchronize()
            assert torch.equal(img, film)
        ref, _ = O.OracleScene(mesh).render(O.reference_params(W, H, spp, D))
        np.testing.assert_array_equal(img.cpu().numpy(), ref)
        # bench.py's max-over-ranks time and summed counters, on the device
        t = torch.tensor([1.25], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tt = torch.tensor([3.0, 5.0, 7.0], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        dist.barrier()
        assert float(t.item()) == 1.25 and tt.tolist() == [3.0, 5.0, 7.0]
    finally:
        dist.destroy_process_group()
