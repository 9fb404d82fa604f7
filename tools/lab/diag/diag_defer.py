"""Deferred slab reductions (library.DEFER_REDUCE): on which thread do the backward ops and
the autograd final callback run, eagerly and under CapturedTrainStep's capture?"""
import sys
import threading
from pathlib import Path

REPO = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd"), str(REPO / "tests")]
import torch  # noqa: E402

from models import library  # noqa: E402

log = []
_orig_flush = library._flush_pending
_orig_rb = library._reduce_batch


def flush():
    log.append(("flush", threading.get_ident(), getattr(library._pending, "batch", None) is not None))
    _orig_flush()


library._flush_pending = flush


def main():
    from helpers import LTA_INP, lta_ids
    from models.detector import LeakDetector
    from models.graph_step import CapturedTrainStep
    from models.loss import CrossEntropyLoss
    from models.optim import ClipAdamW
    import copy
    import contextlib

    @contextlib.contextmanager
    def rb(lib, st, keep=None):
        log.append(("op", threading.get_ident(), getattr(library._pending, "batch", None) is not None))
        with _orig_rb(lib, st, keep):
            yield
    library._reduce_batch = rb
    dev = torch.device("cuda:0")
    sensors, pipes = lta_ids()
    torch.manual_seed(0)
    m1 = LeakDetector(LTA_INP, sensors, pipes, dropout=0.0).to(dev).train()
    m2 = copy.deepcopy(m1)
    gen = torch.Generator().manual_seed(1)
    B = 6
    r = torch.randn(B, 36, 29, generator=gen).to(dev)
    tf = torch.randn(B, 36, 9, generator=gen).to(dev)
    lab = torch.randint(0, len(pipes) + 1, (B,), generator=gen).to(dev)
    print("main thread", threading.get_ident())
    library.DEFER_REDUCE = True
    ce = CrossEntropyLoss()
    m1.zero_grad(set_to_none=True)
    ce(m1(r, tf), lab).backward()
    torch.cuda.synchronize()
    print("eager pass:", log)
    log.clear()
    library.DEFER_REDUCE = False
    o1 = ClipAdamW(m1.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)
    o2 = ClipAdamW(m2.parameters(), lr=1e-3, weight_decay=1e-4, max_norm=1.0)
    import os
    os.environ["LEAKGNN_DEFER_REDUCE"] = "1"
    step = CapturedTrainStep(m2, ce, o2, (r, tf), lab, clip=None, warmup=3)
    print("captured build:", log)

    def eager():
        o1.zero_grad(set_to_none=True)
        loss = ce(m1(r, tf), lab)
        loss.backward()
        o1.step()
        return loss
    for _ in range(3):
        eager()
    for _ in range(4):
        l1 = eager()
        l2 = step()
    torch.cuda.synchronize()
    print("loss", float(l1), float(l2))
    for (n, a), b in zip(m2.named_parameters(), m1.parameters()):
        d = (a - b).abs().max().item()
        if d > 1e-6:
            print("DIFF", n, d)


if __name__ == "__main__":
    main()
