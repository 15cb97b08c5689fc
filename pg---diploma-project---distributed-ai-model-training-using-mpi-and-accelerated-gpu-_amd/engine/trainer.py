"""Training engine: ``Trainer.fit()`` = the reference's epoch loop, re-built.

Reference loops: serial / 1-GPU ``cifar10_serial_mobilenet_224.py:83-153`` and
MPI+DDP ``cifar10_mpi_mobilenet_224.py:156-252``:
per epoch ``set_epoch`` -> train (Adam, CE) -> globally all-reduced train loss
-> eval under ``no_grad`` -> all-reduced test loss -> ``scheduler.step()`` ->
one log line -> keep the best state (by test accuracy) -> save at the end.

Two execution backends share this loop:

* ``hip``   — the MI355X path: device-resident uint8 dataset, fused GPU
  augmentation, static-plan HIP executor, bucketed RCCL all-reduce, fused Adam,
  hipGraph-replayed steps, metrics kept on the device (one host sync per epoch).
* ``torch`` — reference-semantics PyTorch ops (CPU runs, GPU oracle); the same
  flat parameter buffer + bucketed gradient reducer implement data parallelism,
  so the DDP layer is exercised by multi-process CPU (gloo) tests as well.

Metric semantics follow the reference (loss is the global mean, accuracy is
rank-local in the DDP line) and additionally report global accuracy.
"""
import math
import os
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..config import TrainConfig
from ..data.cifar10 import load_dataset
from ..models import build_model
from ..parallel.bootstrap import init_distributed, barrier
from ..parallel.ddp import BucketedGradReducer, broadcast_parameters, all_reduce_scalars
from ..parallel.sampler import ShardSampler
from ..parallel.watchdog import Watchdog
from ..utils import logging as L
from ..utils.profiling import StepTimer, trace_range
from . import checkpoint as ckpt
from .flat import FlatParams


def step_lr(base_lr: float, epoch: int, step_size: int, gamma: float) -> float:
    """torch.optim.lr_scheduler.StepLR value for a 0-based epoch (reference :77, :131)."""
    return base_lr * (gamma ** (epoch // step_size))


class Trainer:
    def __init__(self, cfg: TrainConfig, info=None):
        self.cfg = cfg
        self.info, self.device, self.dist_backend = init_distributed(cfg.dist_backend, cfg.device, info=info,
                                                                     timeout_s=cfg.dist_timeout_s)
        self.rank, self.world = self.info.rank, self.info.world_size
        self.watchdog = None
        if cfg.watchdog_s and cfg.watchdog_s > 0:
            store = None
            try:
                from torch.distributed import distributed_c10d as c10d
                store = c10d._get_default_store() if self.world > 1 else None
            except Exception:
                store = None
            self.watchdog = Watchdog(cfg.watchdog_s, self.rank, self.world, store=store).start()
        self.timer = None
        backend = cfg.backend
        if backend == "auto":
            backend = "hip" if self.device.type == "cuda" else "torch"
        if backend == "hip" and self.device.type != "cuda":
            raise RuntimeError("backend 'hip' needs a GPU")
        self.backend = backend
        self.ddp_log = cfg.log_format == "ddp" or self.world > 1
        if cfg.seed is not None:
            torch.manual_seed(cfg.seed)   # identical init on every rank (reference seeds DDP only)
        self.base_lr = cfg.lr * (self.world if cfg.scale_lr else 1)

        if self.ddp_log:
            for line in L.ddp_banner():
                L.emit(line, self.rank)
            L.emit(L.backend_line(self.dist_backend, self.world, self.device), self.rank)
        else:
            L.emit(L.device_line(self.device), self.rank)

        # ---- data (rank 0 first, then everyone: the reference's download barrier, :93-113)
        if self.rank == 0:
            if self.ddp_log and cfg.data == "cifar10":
                L.emit(L.download_line(), self.rank)
            self.train_data = load_dataset(cfg.data, cfg.data_root, True, cfg.synthetic_train_size,
                                           signal=cfg.synthetic_signal)
        barrier(self.device if self.device.type == "cuda" else None)
        if self.rank != 0:
            self.train_data = load_dataset(cfg.data, cfg.data_root, True, cfg.synthetic_train_size,
                                           signal=cfg.synthetic_signal)
        self.test_data = load_dataset(cfg.data, cfg.data_root, False, cfg.synthetic_test_size,
                                     signal=cfg.synthetic_signal)
        for line in L.samples_lines(len(self.train_data), len(self.test_data)):
            L.emit(line, self.rank)
        self.train_sampler = ShardSampler(len(self.train_data), self.world, self.rank, shuffle=True)
        self.test_sampler = ShardSampler(len(self.test_data), self.world, self.rank, shuffle=False)

        # ---- model
        self.model = build_model(cfg.model, cfg.num_classes, cfg.pretrained)
        L.emit(L.params_line(sum(p.numel() for p in self.model.parameters())), self.rank)
        if backend == "hip":
            self._init_hip()
        else:
            self._init_torch()
        self.start_epoch = 0
        self.best_acc = 0.0
        self.best_state = ckpt.snapshot_state_dict(self.model)   # reference: deepcopy at init
        if cfg.resume:
            self._resume(cfg.resume)

    # ------------------------------------------------------------------ backends
    def _init_hip(self):
        from .native_step import NativeTrainStep
        cfg = self.cfg
        if cfg.model not in ("mobilenet_v2", "resnet50"):
            raise NotImplementedError("native HIP executors: mobilenet_v2, resnet50")
        if cfg.deterministic:
            from ..ops import kernels as K
            K.set_deterministic(True)   # fixed-order BN statistics (bitwise-reproducible runs)
        self.step = NativeTrainStep(self.model, cfg.batch_size, self.device, img_size=cfg.img_size,
                                    lr=self.base_lr, betas=cfg.betas, eps=cfg.eps,
                                    weight_decay=cfg.weight_decay, world_size=self.world, rank=self.rank,
                                    use_graph=cfg.graph, seed=cfg.seed or 0, bucket_mb=cfg.bucket_mb,
                                    first_bucket_mb=cfg.first_bucket_mb,
                                    reduce_dtype=torch.bfloat16 if cfg.grad_reduce_dtype == "bf16" else torch.float32,
                                    augment=True, train_augment=cfg.augment != "none",
                                    bn_broadcast=cfg.bn_sync == "broadcast", fp8=cfg.precision == "fp8",
                                    comm_watchdog_s=cfg.dist_timeout_s if self.world > 1 else None)
        self.flat = self.step.flat
        self.train_src = torch.from_numpy(self.train_data.images).to(self.device)
        self.train_labels = torch.from_numpy(self.train_data.labels).to(self.device)
        self.test_src = torch.from_numpy(self.test_data.images).to(self.device)
        self.test_labels = torch.from_numpy(self.test_data.labels).to(self.device)
        self.step.set_data(self.train_src, self.train_labels)
        self._tail_steps = {}

    def _tail(self, n: int):
        """Training step object for a short last batch (reference DataLoader keeps it: drop_last=False)."""
        if n not in self._tail_steps:
            self._tail_steps[n] = self.step.sibling(n)
        return self._tail_steps[n]

    def _init_torch(self):
        cfg = self.cfg
        dev = self.device
        self.model.to(dev)
        if dev.type == "cuda":
            self.model.to(memory_format=torch.channels_last)
        self.flat = FlatParams(self.model, dev, with_shadow=False)
        if self.world > 1:
            mods = [m for m in self.model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
            broadcast_parameters([self.flat.master] + [b for m in mods for b in (m.running_mean, m.running_var)])
            ranges = [(n,) + self.flat.range_of(n) for n in self.flat.order]
            self.reducer = BucketedGradReducer(self.flat.grad, ranges, cfg.bucket_mb, cfg.first_bucket_mb)
        else:
            self.reducer = None
        params = [self.flat.params[n] for n in self.flat.order]
        self.opt = torch.optim.Adam(params, lr=self.base_lr, betas=cfg.betas, eps=cfg.eps,
                                    weight_decay=cfg.weight_decay)
        self.crit = torch.nn.CrossEntropyLoss()
        self.amp = dev.type == "cuda" and cfg.precision == "bf16"
        self._gen = torch.Generator().manual_seed((cfg.seed or 0) + 1000 * self.rank)

    def _torch_batch(self, data, idx: np.ndarray, train: bool):
        from ..data import augment_torch as A
        imgs = torch.from_numpy(data.images[idx])
        labels = torch.from_numpy(data.labels[idx]).to(self.device)
        if self.cfg.augment == "none" or not train:
            x = A.render(imgs, None, self.cfg.img_size, train=False)
        else:
            prm = A.sample_params(len(idx), self.cfg.img_size, self._gen)
            x = A.render(imgs, prm, self.cfg.img_size, train=True)
        x = x.to(self.device)
        if self.device.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
        return x, labels

    # ------------------------------------------------------------------ epoch pieces
    def set_lr(self, lr: float):
        if self.backend == "hip":
            self.step.set_lr(lr)
        else:
            for g in self.opt.param_groups:
                g["lr"] = lr

    def train_epoch(self, epoch: int):
        """Returns (loss_sum, correct, count) of this rank's shard."""
        self.train_sampler.set_epoch(epoch)
        idx = self.train_sampler.indices()
        bs = self.cfg.batch_size
        nb = math.ceil(len(idx) / bs)
        if self.cfg.max_steps_per_epoch:
            nb = min(nb, self.cfg.max_steps_per_epoch)
        prof = self.cfg.profile
        self.timer = StepTimer(bs * self.world, warmup=2 if epoch == self.start_epoch else 0,
                               device=self.device) if prof else None
        if self.backend == "hip":
            didx = torch.from_numpy(idx).to(self.device)
            self.step.metrics.zero_()
            comm = getattr(self.step, "comm", None)
            with trace_range(f"train_epoch_{epoch}", prof):
                for b in range(nb):
                    # per-step failure check without a host sync: the communicator's error word
                    # copied one step earlier (a failed step's Adam update was skipped on device)
                    if comm is not None and comm.world > 1:
                        err = comm.poll_error()
                        if err:
                            from ..parallel.comm import CommError
                            from ..ops._lib import lib
                            # poison this rank's communicator (device error word included) before
                            # raising, so nothing later on this rank launches a collective
                            lib().comm_poison(comm.id, f"rank {self.rank}: error 0x{err:x} seen by the step poll")
                            raise CommError(f"native communicator error 0x{err:x} on rank {self.rank} before "
                                            f"epoch {epoch + 1} batch {b}: {comm.error_string() or 'P2P failure'}")
                    sl = didx[b * bs:(b + 1) * bs]
                    # the next batch (augmented during this step's backward when it is full-size)
                    nxt = didx[(b + 1) * bs:(b + 2) * bs] if b + 1 < nb else None
                    st = self.step if sl.numel() == bs else self._tail(sl.numel())
                    if self.timer is not None and sl.numel() == bs:
                        self.timer.start()
                        st.run(sl, nxt)
                        self.timer.stop()
                    else:
                        st.run(sl, nxt)
                    if self.watchdog is not None:
                        self.watchdog.kick(phase=f"train epoch {epoch} batch {b}")
                return self.step.read_metrics()
        self.model.train()
        loss_sum, correct, count = 0.0, 0, 0
        for b in range(nb):
            sel = idx[b * bs:(b + 1) * bs]
            x, y = self._torch_batch(self.train_data, sel, True)
            if self.world > 1 and self.cfg.bn_sync == "broadcast":   # DDP broadcast_buffers=True
                broadcast_parameters(self._bn_buffers())
            self.flat.grad.zero_()
            with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
                out = self.model(x)
                loss = self.crit(out.float(), y)
            loss.backward()
            if self.reducer is not None:
                self.reducer.begin()
                self.reducer.mark_ready(self.flat.order)
                self.reducer.finish()
                self.flat.grad.mul_(1.0 / self.world)
            self.opt.step()
            if self.watchdog is not None:
                self.watchdog.kick(phase=f"train epoch {epoch} batch {b}")
            loss_sum += loss.item() * y.numel()
            correct += int((out.argmax(1) == y).sum().item())
            count += y.numel()
        return loss_sum, correct, count

    def _bn_buffers(self):
        mods = [m for m in self.model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
        return [b for m in mods for b in (m.running_mean, m.running_var, m.num_batches_tracked)]

    @torch.no_grad()
    def evaluate(self):
        """Returns (loss_sum, correct, count) over this rank's shard of the test set."""
        if self.world > 1 and self.cfg.bn_sync in ("eval", "broadcast"):
            mods = [m for m in self.model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
            broadcast_parameters([b for m in mods for b in (m.running_mean, m.running_var)])
        idx = self.test_sampler.indices()
        bs = self.cfg.batch_size
        if self.backend == "hip":
            from ..ops import kernels as K
            exe = self.step.exe
            exe.eval_prepare()
            didx = torch.from_numpy(idx).to(self.device)
            acc = torch.zeros(3, dtype=torch.float64, device=self.device)
            for s in range(0, len(idx), bs):
                sl = didx[s:s + bs]
                n = sl.numel()
                if n < bs:   # pad: eval BN uses running stats, so rows are independent
                    sl = torch.cat([sl, sl[:1].expand(bs - n)])
                self.step.idx.copy_(sl)
                K.augment(self.test_src, self.step.idx, self.test_labels, exe.img, exe.labels,
                          self.step.aug_params, train=False, double_resize=True, out_hw=self.cfg.img_size)
                exe.forward(train=False)
                acc[0] += exe.loss[:n].double().sum()
                acc[1] += exe.correct[:n].double().sum()
                acc[2] += n
            return acc.tolist()
        self.model.eval()
        loss_sum, correct, count = 0.0, 0, 0
        for s in range(0, len(idx), bs):
            x, y = self._torch_batch(self.test_data, idx[s:s + bs], False)
            with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
                out = self.model(x)
            loss_sum += F.cross_entropy(out.float(), y, reduction="sum").item()
            correct += int((out.argmax(1) == y).sum().item())
            count += y.numel()
        return loss_sum, correct, count

    # ------------------------------------------------------------------ loop
    def fit(self):
        cfg = self.cfg
        L.emit("Starting distributed training...\n" if self.ddp_log else "Starting serial training...", self.rank)
        total = time.time()
        history = []
        for epoch in range(self.start_epoch, cfg.epochs):
            t0 = time.time()
            lr = step_lr(self.base_lr, epoch, cfg.step_size, cfg.gamma)
            self.set_lr(lr)
            tl, tc, tn = self.train_epoch(epoch)
            # native communicator health, once per epoch on every rank (collective): a peer
            # timeout, an out-of-step peer or an RCCL error on ANY rank raises on EVERY rank
            # instead of training on with un-reduced gradients
            comm = getattr(self.step, "comm", None) if self.backend == "hip" else None
            if comm is not None:
                comm.check_all()
            g_tl, g_tn, g_tc = all_reduce_scalars([tl, tn, tc], self.device)
            train_loss = g_tl / max(g_tn, 1)
            train_acc_local = tc / max(tn, 1)
            if cfg.eval_every and ((epoch + 1) % cfg.eval_every == 0 or epoch + 1 == cfg.epochs):
                el, ec, en = self.evaluate()
                g_el, g_en, g_ec = all_reduce_scalars([el, en, ec], self.device)
                test_loss = g_el / max(g_en, 1)
                test_acc_local = ec / max(en, 1)
                test_acc_global = g_ec / max(g_en, 1)
            else:
                test_loss = test_acc_local = test_acc_global = float("nan")
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            dt = time.time() - t0
            if self.ddp_log:
                L.emit(L.ddp_epoch_line(epoch + 1, cfg.epochs, dt, train_loss, test_loss, test_acc_local), self.rank)
            else:
                L.emit(L.serial_epoch_line(epoch + 1, cfg.epochs, dt, train_loss, train_acc_local, test_loss,
                                           test_acc_local), self.rank)
            if self.timer is not None:
                t = self.timer.summary()
                if t.get("steps"):
                    L.emit(f"[pgdist] epoch {epoch + 1} step {t['mean_ms']:.2f} ms (p50 {t['p50_ms']:.2f}, "
                           f"p90 {t['p90_ms']:.2f}) -> {t['img_per_s']:.0f} img/s (train steps only)", self.rank)
            if self.watchdog is not None:
                self.watchdog.kick(phase=f"epoch {epoch + 1} done")
            if cfg.global_accuracy and self.world > 1:
                L.emit(f"[pgdist] epoch {epoch + 1} global test acc {test_acc_global:.4f} "
                       f"train img/s {g_tn / dt:.1f}", self.rank)
            history.append(dict(epoch=epoch + 1, time=dt, train_loss=train_loss, train_acc=train_acc_local,
                                test_loss=test_loss, test_acc=test_acc_local, test_acc_global=test_acc_global,
                                lr=lr, train_images=g_tn))
            # best model by (rank-local) test accuracy, like the reference (:143-145 / :238-240)
            if test_acc_local == test_acc_local and test_acc_local > self.best_acc:
                self.best_acc = test_acc_local
                self.best_state = ckpt.snapshot_state_dict(self.model)
            if cfg.ckpt_dir and self.rank == 0:
                self._save_full(epoch + 1, lr)
            if cfg.ckpt_dir and self.world > 1:
                # the peers wait here (host barrier, dist_timeout_s) while rank 0 writes the
                # checkpoint, not inside the next epoch's first collective, where the native
                # communicator's watchdog would see a stall
                barrier(self.device if self.device.type == "cuda" else None)
        total = time.time() - total
        if self.world > 1:
            self.replica_check()
        L.emit("", self.rank)
        L.emit(L.best_line(self.best_acc, self.ddp_log), self.rank)
        L.emit(L.total_time_line(total), self.rank)
        save_path = cfg.save_path or ("best_mobilenetv2_cifar10_224_mpi.pth" if self.ddp_log
                                      else "best_mobilenetv2_cifar10_224.pth")
        if self.rank == 0 and save_path:
            ckpt.save_best(self.best_state, save_path)
            L.emit(L.saved_line(save_path), self.rank)
        self.history = history
        if self.watchdog is not None:
            self.watchdog.stop()
        return history

    def replica_check(self):
        """Data-parallel consistency: parameters (and, with bn_sync eval/broadcast, the BN running
        statistics that evaluation synchronises) must be bitwise identical on every rank."""
        from ..parallel.ddp import replicas_identical
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        params = [self.step.flat.master] if self.backend == "hip" else \
            [p for p in self.model.parameters()]
        ok_p, dp = replicas_identical(params, self.device)
        bufs = self._bn_buffers()
        ok_b, db = replicas_identical(bufs, self.device)
        self.replicas_ok = (ok_p, ok_b)
        L.emit(f"[pgdist] replica check over {self.world} ranks: parameters "
               f"{'identical' if ok_p else 'DIFFER'} (digest {int(dp[0]):x}), BN buffers "
               f"{'identical' if ok_b else 'DIFFER'} (digest {int(db[0]):x}, bn_sync={self.cfg.bn_sync})",
               self.rank)
        # the verdict is the same on every rank (MIN == MAX of the digests), so every rank raises
        bn_synced = self.cfg.bn_sync in ("eval", "broadcast") and bool(self.cfg.eval_every)
        if not ok_p or (bn_synced and not ok_b):
            raise RuntimeError(f"data-parallel replicas diverged over {self.world} ranks: parameters "
                               f"{'identical' if ok_p else 'DIFFER'}, BN buffers {'identical' if ok_b else 'DIFFER'}")

    # ------------------------------------------------------------------ checkpoint/resume
    def _adam_step(self) -> int:
        if self.backend == "hip":
            return int(self.step.hyper[1].item())
        st = self.opt.state.get(self.flat.params[self.flat.order[0]], {})
        return int(st.get("step", 0))

    def _save_full(self, epoch: int, lr: float):
        if self.backend == "hip":
            m, v = self.flat.exp_avg, self.flat.exp_avg_sq
        else:
            m = torch.zeros_like(self.flat.master)
            v = torch.zeros_like(self.flat.master)
            for n in self.flat.order:
                st = self.opt.state.get(self.flat.params[n], {})
                if "exp_avg" in st:
                    self.flat.view(m, n, st["exp_avg"].shape).copy_(st["exp_avg"])
                    self.flat.view(v, n, st["exp_avg_sq"].shape).copy_(st["exp_avg_sq"])
        path = os.path.join(self.cfg.ckpt_dir, f"ckpt_epoch{epoch}.pt")
        ckpt.save_full(path, model=self.model, epoch=epoch, step=self._adam_step(), lr=lr, exp_avg=m,
                       exp_avg_sq=v, flat_order=self.flat.order, best_acc=self.best_acc,
                       best_state=self.best_state, world_size=self.world,
                       config={k: (list(v) if isinstance(v, tuple) else v) for k, v in vars(self.cfg).items()})

    def _resume(self, path: str):
        if path == "auto":
            path = ckpt.latest_checkpoint(self.cfg.ckpt_dir)
            if path is None:
                return
        obj = ckpt.load_full(path)
        self.model.load_state_dict(obj["model"])
        if obj["flat_order"] != self.flat.order:
            raise RuntimeError("checkpoint parameter layout does not match this model")
        if self.backend == "hip":
            self.flat.exp_avg.copy_(obj["exp_avg"].to(self.device))
            self.flat.exp_avg_sq.copy_(obj["exp_avg_sq"].to(self.device))
            self.step.hyper[1:2].fill_(float(obj["step"]))
            self.flat.refresh_shadow()
        else:
            m, v = obj["exp_avg"].to(self.device), obj["exp_avg_sq"].to(self.device)
            for n in self.flat.order:
                p = self.flat.params[n]
                self.opt.state[p] = {"step": torch.tensor(float(obj["step"])),
                                     "exp_avg": self.flat.view(m, n, p.shape).clone(),
                                     "exp_avg_sq": self.flat.view(v, n, p.shape).clone()}
        self.start_epoch = int(obj["epoch"])
        self.best_acc = float(obj["best_acc"])
        if obj.get("best_state"):
            self.best_state = obj["best_state"]
        L.emit(f"[pgdist] resumed from {path} at epoch {self.start_epoch}", self.rank)
