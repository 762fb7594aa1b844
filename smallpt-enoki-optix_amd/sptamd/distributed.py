"""Multi-GPU image tiling + framebuffer gather (one process per GPU).

Each rank renders the interleaved row-group tile `rank` of `world`
(spt_render_params.tile_*), then the fp32 tiles (3 x rows x W, padded to the
largest tile) are gathered to rank 0 with ONE collective — torch.distributed
gather, i.e. RCCL over xGMI on the nccl backend — and rank 0 scatters the rows
back into the full image.  The reference is single-GPU (no collective,
SURVEY §2); this is the build's only exchange step.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ._lib import tile_rows


class TileGather:
    def __init__(self, height: int, width: int, rank: int, world: int, rows_per_group: int,
                 device: torch.device):
        self.H, self.W, self.rank, self.world = height, width, rank, world
        self.rows: List = [tile_rows(height, r, world, rows_per_group) for r in range(world)]
        self.max_rows = max(1, max(len(r) for r in self.rows))
        self.device = device
        # flat so that every rank's (3, rows, W) film is one contiguous prefix;
        # two of them, so that consecutive steps can render on two streams
        # while the previous step's tile is still being gathered
        self.tiles = [torch.zeros(3 * self.max_rows * width, dtype=torch.float32, device=device)]
        self.tile = self.tiles[0]
        self.gather_list: Optional[List[torch.Tensor]] = None
        self.image: Optional[torch.Tensor] = None
        # the collective runs whenever a process group exists (at world size
        # 1 too: one rank's RCCL gather), else one process copies its tile
        self.collective = world > 1 or (dist.is_available() and dist.is_initialized())
        if rank == 0:
            self.image = torch.zeros((3, height, width), dtype=torch.float32, device=device)
            self.row_index = [torch.as_tensor(r, dtype=torch.long, device=device) for r in self.rows]
            if self.collective:
                self.gather_list = [torch.empty_like(self.tile) for _ in range(world)]

    @property
    def my_rows(self) -> int:
        return len(self.rows[self.rank])

    def tile_view(self, k: int = 0) -> torch.Tensor:
        """The (3, my_rows, W) film buffer k (0 or 1) spt_render writes into."""
        while len(self.tiles) <= k:
            self.tiles.append(torch.zeros_like(self.tiles[0]))
        return self.tiles[k][: 3 * self.my_rows * self.W].view(3, self.my_rows, self.W)

    def gather(self, k: int = 0) -> Optional[torch.Tensor]:
        """Collective: every rank calls it; rank 0 gets the assembled image
        from every rank's film buffer k (on the current stream)."""
        tile = self.tiles[k]
        if not self.collective:
            self.image.copy_(self.tile_view(k))
            return self.image
        if tile.is_cuda and dist.get_backend() != "nccl":
            # gloo gathers host tensors only (the CPU rehearsal of the N-rank flow)
            tile = tile.cpu()
            glist = [torch.empty_like(tile) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(tile, glist, dst=0)
            if self.rank == 0:
                for r in range(self.world):
                    self.gather_list[r].copy_(glist[r])
        else:
            dist.gather(tile, self.gather_list if self.rank == 0 else None, dst=0)
        if self.rank != 0:
            return None
        for r in range(self.world):
            n = len(self.rows[r])
            if n:
                self.image[:, self.row_index[r], :] = self.gather_list[r][: 3 * n * self.W].view(3, n, self.W)
        return self.image
