"""N>1 path on CPU: world_size-2, 3 and 8 gloo processes, each renders its interleaved
row-group tile (with the CPU oracle standing in for the GPU renderer) and the
package's TileGather gathers and assembles the framebuffer on rank 0; the
result must equal the single-process render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP, DEPTH = 24, 19, 2, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, rpg, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "smallpt-enoki-optix_amd"), os.path.join(root, "oracle")]
    import oracle as O
    from sptamd import scenes
    from sptamd.distributed import TileGather

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mesh = scenes.mitsuba_synth(detail=0.1)
        tg = TileGather(H, W, rank, world, rpg, torch.device("cpu"))
        film, _ = O.OracleScene(mesh).render(O.reference_params(W, H, SPP, DEPTH), rows=tg.rows[rank], nthreads=2)
        tg.tile_view().copy_(torch.from_numpy(film))
        img = tg.gather()
        if rank == 0:
            np.save(out_path, img.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rpg", [(2, 1), (2, 4), (3, 8), (8, 1), (8, 2)])
def test_tile_gather_matches_single_render(tmp_path, world, rpg):
    import oracle as O
    from sptamd import scenes

    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), rpg, out), nprocs=world, join=True)
    full, _ = O.OracleScene(scenes.mitsuba_synth(detail=0.1)).render(O.reference_params(W, H, SPP, DEPTH))
    np.testing.assert_array_equal(np.load(out), full)


def test_tile_rows_partition():
    import sptamd
    for world in (1, 2, 3, 8):
        for rpg in (1, 5, 8, 128):
            rows = [sptamd.tile_rows(1000, r, world, rpg) for r in range(world)]
            allr = np.sort(np.concatenate(rows))
            np.testing.assert_array_equal(allr, np.arange(1000))
            for r, rr in enumerate(rows):
                assert np.all(((rr // rpg) % world) == r)
