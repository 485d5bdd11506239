"""Data-parallel training semantics on CPU (gloo, world_size 2).

Two ranks, each holding half of every micro-batch, must end with the same parameters (and EMA) as one
process holding the whole micro-batch. This covers the whole Phase-6 optimizer step: accumulation,
FGM with the globally reduced direction, clip 3.0, AdamW, EMA and warmup+cosine. Mixup is off
because it permutes within a micro-batch, so splitting the batch changes its pairs. The loss is
focal with a plain mean (Phase 6). The weighted-CE fallback's mean is normalised by the batch's
class weights, so it is not rank-decomposable (and the reference has no data-parallel mode).
`radhip.train.fgm_attack` (the HIP kernel) is swapped for the same update written in torch, since a
CPU box cannot run the kernel. The kernel itself is checked in tests/test_kernels_gpu.py.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.feature_projection = torch.nn.Linear(6, 5)
        self.body = torch.nn.Linear(5, 4)
        self.classifier = torch.nn.Linear(4, 2)

    def forward(self, x, Freq_aug=False):
        h = torch.tanh(self.body(torch.tanh(self.feature_projection(x))))
        return h, self.classifier(h)


# Phase-6 loss: focal with a plain batch mean, which decomposes over ranks. The weighted-CE fallback
# does not: its mean divides by the batch's sum of class weights.
CFG = {"loss": "Focal", "freq_aug": "False",
       "optim_config": {"base_lr": 5e-3, "wavlm_lr": 1e-2, "weight_decay": 1e-4, "scheduler": "cosine",
                        "scheduler_config": {"eta_min": 1e-6}},
       "training_config": {"use_mixup": False, "accumulation_steps": 2, "use_ema": True, "ema_decay": 0.9,
                           "use_fgm": True, "fgm_epsilon": 0.5, "warmup_steps": 1, "warmup_init_factor": 0.1,
                           "freeze_bn": True, "focal_alpha": 0.9, "focal_gamma": 2.5}}


def _torch_fgm(params, grads, backups, eps):
    """Same update as rdx_fgm_attack: backup, then p += eps * g / ||g|| (skip zero/NaN norms)."""
    for p, g, b in zip(params, grads, backups):
        b.copy_(p)
        nrm = torch.linalg.vector_norm(g.double())
        if nrm != 0 and not torch.isnan(nrm):
            p.add_((eps * g.double() / nrm).to(p.dtype))


def _train(rank, world, xs, ys, init):
    import radhip.train as T
    T.fgm_attack = _torch_fgm
    torch.manual_seed(0)
    m = Toy()
    m.load_state_dict(init)
    groups = [{"params": list(m.feature_projection.parameters()), "lr": 1e-2},
              {"params": list(m.body.parameters()) + list(m.classifier.parameters()), "lr": 5e-3}]
    tr = T.Trainer(m, CFG, "cpu", total_steps=3, amp_dtype=torch.float32, param_groups=groups)
    n_micro, B = xs.shape[0], xs.shape[1]
    sl = slice(rank * B // world, (rank + 1) * B // world)
    for i in range(n_micro):
        x = torch.from_numpy(xs[i][sl])
        tr.micro_step(x, torch.from_numpy(ys[i][sl]), last_in_epoch=(i == n_micro - 1))
    params = {k: v.detach().clone() for k, v in m.state_dict().items()}
    ema = tr.ema.state_dict()
    return params, ema


def _worker(rank, world, port, xs, ys, init, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params, ema = _train(rank, world, xs, ys, init)
        torch.save({"params": params, "ema": ema}, os.path.join(out, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_training_equals_single_process():
    rng = np.random.default_rng(3)
    xs = rng.standard_normal((6, 4, 6)).astype(np.float32)      # 6 micro-batches of 4
    ys = rng.integers(0, 2, (6, 4)).astype(np.int64)
    torch.manual_seed(1)
    init = {k: v.clone() for k, v in Toy().state_dict().items()}
    ref_params, ref_ema = _train(0, 1, xs, ys, init)
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(2, _free_port(), xs, ys, init, out), nprocs=2, join=True,
                           start_method="spawn")
        got = [torch.load(os.path.join(out, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    for r in range(2):
        for k, v in ref_params.items():
            torch.testing.assert_close(got[r]["params"][k], v, rtol=2e-5, atol=1e-6, msg=f"rank{r} {k}")
        for k, v in ref_ema.items():
            torch.testing.assert_close(got[r]["ema"][k], v, rtol=2e-5, atol=1e-6, msg=f"rank{r} ema {k}")
    # the ranks agree bit-for-bit with each other (identical all-reduced grads)
    for k in ref_params:
        assert torch.equal(got[0]["params"][k], got[1]["params"][k]), k


def test_fgm_direction_uses_global_gradient():
    """With FGM on, a rank's attack must use the sum of all ranks' accumulated grads."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_fgm_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
        got = [torch.load(os.path.join(out, f"g{r}.pt"), weights_only=True) for r in range(2)]
    want = torch.tensor([1.0, 2.0, 3.0]) + torch.tensor([-4.0, 0.5, 2.0])
    for g in got:
        torch.testing.assert_close(g, want)


def _fgm_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from radhip.train import fgm_global_grads
        g = [torch.tensor([1.0, 2.0, 3.0]) if rank == 0 else torch.tensor([-4.0, 0.5, 2.0])]
        torch.save(fgm_global_grads(g)[0], os.path.join(out, f"g{rank}.pt"))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
