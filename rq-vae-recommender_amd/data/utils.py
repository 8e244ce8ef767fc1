"""Loader helpers (reference data/utils.py:4-16). batch_to copies host batches to the device
with non_blocking transfers (pinned sources overlap the H2D copy with compute)."""
from data.schemas import SeqBatch


def cycle(dataloader):
    while True:
        for data in dataloader:
            yield data


def batch_to(batch, device):
    return SeqBatch(*[v.to(device, non_blocking=True) if hasattr(v, "to") else v for _, v in batch._asdict().items()])


def next_batch(dataloader, device):
    batch = next(dataloader)
    return batch_to(batch, device)
