"""DataLoader construction with exactly-once sharding across data-parallel ranks.

The reference builds a DistributedSampler AND lets accelerate re-shard the loader, so each rank
sees 1/world^2 of the data per epoch. Here the sampler is the only
sharding layer."""
from __future__ import annotations

from typing import Optional

import torch
from torch.utils.data import DataLoader, DistributedSampler

from ..parallel.dist import state as dist_state


def get_distributed_sampler(dataset, shuffle: bool = True, seed: int = 0, drop_last: bool = False):
    """Shard over DATA-parallel replicas: under tensor parallelism every rank of a TP group must
    see the same samples, so the replica index is the mesh's dp_rank, not the global rank."""
    from ..parallel.mesh import current_mesh

    st = dist_state()
    mesh = current_mesh()
    n, r = (mesh.dp, mesh.dp_rank) if mesh is not None else (st.world_size, st.rank)
    if n > 1 or shuffle:
        # also for one replica: the epoch-seeded permutation makes a resumed run see exactly
        # the batches the interrupted run would have (set_epoch + skip in train_loop)
        return DistributedSampler(dataset, num_replicas=n, rank=r, shuffle=shuffle,
                                  seed=seed, drop_last=drop_last)
    return None


def build_dataloader(dataset, batch_size: int, shuffle: bool = True, num_workers: int = 0,
                     seed: int = 0, collate_fn=None, drop_last: bool = False,
                     pin_memory: Optional[bool] = None):
    sampler = get_distributed_sampler(dataset, shuffle=shuffle, seed=seed, drop_last=drop_last)
    g = torch.Generator()
    g.manual_seed(seed)
    return DataLoader(dataset, batch_size=batch_size, sampler=sampler,
                      shuffle=(shuffle and sampler is None), num_workers=num_workers,
                      collate_fn=collate_fn or getattr(dataset, "collate", None), drop_last=drop_last,
                      pin_memory=torch.cuda.is_available() if pin_memory is None else pin_memory,
                      generator=g if sampler is None else None,
                      persistent_workers=num_workers > 0), sampler
