"""Training program with the reference's semantics (``run.py:121-325``).

Kept from the reference (parity): flag names/defaults, Kinetics layout and clip sampling, transform
math, cosine schedule length ``(len(global train loader) * epochs) // gas`` stepped at the global rate,
loss ``/ gas``, optimizer boundary ``step % gas == 0`` (first optimizer step after one micro-batch),
log keys (``train_loss_step``, ``lr`` every ``log_every``; ``accuracy``, ``train_loss_epoch``, ``epoch``
per epoch), checkpoint directory names ``step_{global_step}`` / ``epoch_{e}`` and resume parsing,
``limit_*_batches`` (break at ``step == limit`` ⇒ limit+1 batches), per-GPU BatchNorm statistics.

Deliberately fixed (README, "Differences from the reference"):
* integer ``--checkpointing_steps`` (Fire parses ``1000`` as int) is honoured (R7a);
* ``--seed`` is honoured instead of the hard-coded 42 (R7b);
* ``--resume_from_checkpoint latest`` resumes from the newest ``epoch_*``/``step_*`` (R7k dead branch);
  ``global_step`` continues from the checkpoint instead of restarting at 0; skipped batches are not
  decoded;
* datasets have exact lengths and validation covers every uniform clip (R2);
* the final save no longer raises ``UnboundLocalError`` without checkpointing (R7r): it goes to
  ``<output_dir>/final``;
* gradients are all-reduced once per optimizer step (``no_sync`` on the other micro-steps; math-identical);
  BN running statistics are broadcast from rank 0 before evaluation and saving instead of every forward;
  validation accuracy is one counter all-reduce per epoch instead of two all-gathers per batch.
"""
from __future__ import annotations

import math
import os
import time
from argparse import Namespace
from typing import Optional

import torch

from ..data.kinetics import LabeledVideoPaths, SyntheticVideoPaths, VideoClipDataset
from ..models import reference as R
from ..utils.misc import set_seed
from ..utils.metrics import Accuracy
from ..utils.profiling import StepTimer
from ..utils.progress import progress_bar
from .accelerator import Accelerator


class InjectedFault(RuntimeError):
    """Raised by ``PVA_FAULT=step=N`` (fault-injection test hook for elastic restarts)."""


def _maybe_inject_fault(global_step: int, output_dir: str):
    """``PVA_FAULT=step=N``: fail once when global step N completes (a marker file in ``output_dir``
    makes the restarted run pass through)."""
    from ..utils.misc import fault_at
    at = fault_at("step")
    if at is None or global_step != at:
        return
    marker = os.path.join(output_dir or ".", f".fault_injected_{os.environ.get('RANK', '0')}")
    if os.path.exists(marker):
        return
    os.makedirs(os.path.dirname(marker), exist_ok=True)
    open(marker, "w").close()
    raise InjectedFault(f"injected fault at global step {global_step}")


def parse_checkpointing_steps(v):
    if v is None:
        return None
    if isinstance(v, bool):
        raise ValueError("checkpointing_steps must be an int or 'epoch'")
    if isinstance(v, int):
        return v
    if isinstance(v, str):
        if v == "epoch":
            return "epoch"
        if v.isdigit():
            return int(v)
    raise ValueError(f"Argument `checkpointing_steps` must be either a number or `epoch`. `{v}` passed.")


def build_model(args, num_labels: int) -> torch.nn.Module:
    """Hub architecture (slowfast_r50 / slowfast_r101 / slow_r50) + replaced head (reference run.py:105-118)."""
    name = getattr(args, "model", None) or ("slowfast_r50" if args.is_slowfast else "slow_r50")
    # hub pools are 7x7 (final map of a 224 crop); clamp for smaller crops so tiny configs still run
    hs = min(7, max(1, args.crop_size // 32))
    if name.startswith("slowfast"):
        depth = 101 if name.endswith("101") else 50
        net = R.create_slowfast(depth, 400, alpha=args.slowfast_alpha,
                                head_pool_kernel_sizes=((args.num_frames // args.slowfast_alpha, hs, hs),
                                                        (args.num_frames, hs, hs)))
        in_f = 2304
    else:
        net = R.create_resnet(50, 400, head_pool_kernel_size=(args.num_frames, 7, 7))
        in_f = 2048
    if args.pretrained:
        path = getattr(args, "pretrained_path", None) or os.environ.get("PVA_PRETRAINED")
        if path and os.path.exists(path):
            sd = torch.load(path, map_location="cpu", weights_only=True)
            sd = sd.get("model_state", sd) if isinstance(sd, dict) else sd
            missing, unexpected = net.load_state_dict(sd, strict=False)
            print(f"loaded pretrained weights from {path} (missing {len(missing)}, unexpected {len(unexpected)})")
        else:
            print("warning: --pretrained requested but no local weights (--pretrained_path / PVA_PRETRAINED); "
                  "the hub download needs network access — continuing from random init")
    net.blocks[:-1].requires_grad_(not args.freeze_backbone)
    if name.startswith("slowfast"):
        net.blocks[-1] = R.create_res_basic_head(in_f, num_labels, pool=None)
    else:
        net.blocks[-1] = R.create_res_basic_head(in_f, num_labels, pool="default", pool_kernel_size=(1, hs, hs))
    return net


def _datasets(args, acc: Accelerator, mode: str):
    clip_duration = (args.sampling_rate * args.num_frames) / args.frames_per_second
    if args.synthetic:
        mf = getattr(args, "synthetic_min_frames", None)
        train_v = SyntheticVideoPaths(args.synthetic_videos, args.synthetic_classes, seed=1, min_frames=mf)
        val_v = SyntheticVideoPaths(max(args.synthetic_videos // 4, 1), args.synthetic_classes, seed=2, min_frames=mf)
    else:
        train_v = LabeledVideoPaths.from_directory(os.path.join(args.data_dir, "train"))
        val_v = LabeledVideoPaths.from_directory(os.path.join(args.data_dir, "val"))
    common = dict(num_frames=args.num_frames, crop_size=args.crop_size,
                  slowfast_alpha=args.slowfast_alpha if args.is_slowfast else None, rank=acc.process_index,
                  world=acc.num_processes, distributed=acc.num_processes > 1, seed=args.seed, mode=mode)
    train = VideoClipDataset(train_v, clip_duration, True, **common)
    val = VideoClipDataset(val_v, clip_duration, False, full_val=not args.reference_val, **common)
    return train_v, train, val


class _CpuBatches:
    """CPU/torch-backend loader: DataLoader over float clips (reference transform on the host)."""

    def __init__(self, ds, batch_size, num_workers, pin):
        from ..data.loader import make_host_loader
        self.ds = ds
        self.dl = make_host_loader(ds, batch_size, num_workers, pin)

    def __len__(self):
        return len(self.dl)

    def __iter__(self):
        for b in self.dl:
            yield {"video": b["video"], "label": b["label"]}


def training_function(args: Namespace) -> dict:
    checkpointing_steps = parse_checkpointing_steps(args.checkpointing_steps)
    acc = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision, log_with="all",
                      logging_dir=args.logging_dir, kernels=args.kernels)
    set_seed(args.seed)
    mode = "gpu" if acc.kernels == "fused" else "cpu"
    train_videos, train_ds, val_ds = _datasets(args, acc, mode)
    num_labels = train_videos.num_labels

    model = build_model(args, num_labels)
    backend = acc.prepare_model(model)
    if mode == "gpu":
        from ..data.loader import DeviceLoader, make_host_loader
        from ..data.transforms import GpuClipBatch
        prep = GpuClipBatch(acc.device, args.num_frames, args.crop_size,
                            args.slowfast_alpha if args.is_slowfast else None, s2d=backend.net.input_s2d,
                            dtype=backend.net.cdt)
        train_loader = DeviceLoader(make_host_loader(train_ds, args.batch_size, args.num_workers, args.pin_memory),
                                    prep, acc.device)
        val_loader = DeviceLoader(make_host_loader(val_ds, args.batch_size, args.num_workers, args.pin_memory),
                                  prep, acc.device)
    else:
        train_loader = _CpuBatches(train_ds, args.batch_size, args.num_workers, args.pin_memory)
        val_loader = _CpuBatches(val_ds, args.batch_size, args.num_workers, args.pin_memory)

    optimizer = acc.make_optimizer(backend, args.lr, args.momentum, args.weight_decay)
    if args.freeze_backbone:
        # only the replaced head trains: restrict the fused step to its span of the flat buffer
        lo = 0
        hi = max(backend.flat.span(p)[1] for p in model.blocks[-1].parameters())
        optimizer.span = (lo, hi)
        backend.sync.restrict(lo, hi)
    global_batches = math.ceil(train_videos.num_videos / args.batch_size)  # len(train_loader) before prepare
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(
        optimizer, (global_batches * args.num_epochs) // args.gradient_accumulation_steps, last_epoch=-1)
    scheduler = acc.prepare_scheduler(sched, optimizer)
    acc.register_for_checkpointing(scheduler)

    steps_per_epoch = len(train_loader)
    global_step = 0
    starting_epoch = 0
    resume_step = None
    resume = args.resume_from_checkpoint
    if not resume and os.environ.get("PVA_AUTO_RESUME") == "1":
        # elastic restart (launch.py --auto_resume): continue from the newest checkpoint if there is one
        from ..ckpt.state import latest_checkpoint
        resume = latest_checkpoint(args.output_dir or ".") or None
    if resume:
        if resume == "latest":
            from ..ckpt.state import latest_checkpoint
            resume = latest_checkpoint(args.output_dir or ".")
        if resume:
            acc.print(f"Resumed from checkpoint: {resume}")
            acc.load_state(resume)
            diff = os.path.splitext(os.path.basename(os.path.normpath(resume)))[0]
            acc.print("\nTRAINING DIFFERENCE", diff)
            if "epoch" in diff:
                starting_epoch = int(diff.replace("epoch_", "")) + 1
                global_step = starting_epoch * steps_per_epoch
            else:
                n = int(diff.replace("step_", ""))
                starting_epoch = n // max(steps_per_epoch, 1)
                resume_step = n - starting_epoch * steps_per_epoch
                global_step = n

    if args.with_tracking:
        run = str(args.logging_dir).replace(".", "").replace("/", "").replace("\\", "")
        acc.print(f"Initializing tracker for run {run}")
        # the precision / execution path that actually runs is part of the logged config (auditable runs)
        acc.init_trackers(run, {**vars(args), "compute_dtype": acc.compute_dtype, "backend": backend.name})

    gas = args.gradient_accumulation_steps
    history = {"train_loss_epoch": [], "accuracy": [], "clips_per_sec": [], "perf": [],
               "compute_dtype": acc.compute_dtype, "backend": backend.name}
    timer = StepTimer(acc.device)
    backend.timer = timer
    val_metric = Accuracy(acc.device, acc.state)
    output_dir = None
    show = acc.is_main_process and not getattr(args, "quiet", False)
    # reference run.py:233: one bar over every epoch's steps, main process only
    bar = progress_bar(args.num_epochs * steps_per_epoch, disable=not show)
    if global_step:
        bar.update(min(global_step, args.num_epochs * steps_per_epoch))
    for epoch in range(starting_epoch, args.num_epochs):
        bar.set_description_str("Epoch: %s" % epoch)
        train_ds.set_epoch(epoch)
        backend.train()
        total_loss = torch.zeros((), device=acc.device)
        t0, clips = time.perf_counter(), 0
        skip = resume_step if (epoch == starting_epoch and resume_step) else 0
        if skip:
            # skip without decoding: drop the first `skip` batches of the epoch plan
            train_ds.items = train_ds.items[skip * args.batch_size:]
        it = iter(train_loader)
        # steps this epoch runs (limit_train_batches breaks at step == limit), for reading the validation set's
        # first batches ahead of the end of training
        n_run = min(steps_per_epoch - skip, args.limit_train_batches + 1 - skip) if args.limit_train_batches >= 0 \
            else steps_per_epoch - skip
        i = -1
        while True:
            timer.begin_step()
            with timer.host("data"):
                batch = next(it, None)
            if batch is None:
                timer._cur = None
                break
            i += 1
            step = i + skip
            boundary = step % gas == 0
            loss, _ = backend.train_step(batch["video"], batch["label"], 1.0 / gas, sync=boundary)
            if boundary:
                with timer.phase("opt"):
                    sc = getattr(backend, "scaler", None)
                    if sc is not None:
                        scale0 = sc.get_scale()
                        sc.step(optimizer)
                        sc.update()
                        optimizer.step_was_skipped = sc.get_scale() < scale0
                    else:
                        optimizer.step()
                    scheduler.step()
                    optimizer.zero_grad()
            timer.end_step(batch["label"].shape[0] * acc.num_processes)
            bar.update(1)
            global_step += 1
            acc.step = global_step
            clips += batch["label"].shape[0] * acc.num_processes
            step_loss = loss.detach().float() / gas
            if args.with_tracking:
                total_loss += step_loss
                if (step + 1) % args.log_every == 0:
                    perf = timer.summary()
                    history["perf"].append(perf)
                    acc.log({"train_loss_step": step_loss.item(), "lr": optimizer.param_groups[0]["lr"], **perf},
                            step=global_step)
            if show and (step + 1) % max(args.log_every, 1) == 0:
                bar.set_postfix_str(f"loss {step_loss.item():.4f} lr {optimizer.param_groups[0]['lr']:.5f}")
            if isinstance(checkpointing_steps, int) and global_step % checkpointing_steps == 0:
                output_dir = os.path.join(args.output_dir or ".", f"step_{global_step}")
                acc.save_state(output_dir)
                acc.print(f"Saving checkpoint to {output_dir}")
            _maybe_inject_fault(global_step, args.output_dir)
            if i + 3 >= n_run and hasattr(val_loader, "start"):
                val_loader.start()
            if step == args.limit_train_batches:
                break
        if hasattr(it, "close"):   # a loop left at limit_train_batches: stop its reader now, not at collection
            it.close()
        if acc.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        history["clips_per_sec"].append(clips / max(dt, 1e-9))
        if skip:
            train_ds.set_epoch(epoch, force=True)
        if epoch + 1 < args.num_epochs and hasattr(train_loader, "start"):
            # the next epoch's first batches are read while this epoch's validation runs
            train_ds.set_epoch(epoch + 1)
            train_loader.start()

        # ---------------- evaluation
        bar.set_description_str("Val Epoch: %s" % epoch)
        acc.sync_buffers()
        backend.eval()
        val_metric.reset()
        for step, batch in enumerate(val_loader):
            logits = backend.eval_step(batch["video"])
            if hasattr(backend, "eval_counts"):    # fused path: argmax + count on device
                val_metric.update_counts(backend.eval_counts(logits, batch["label"]))
            else:
                val_metric.update(logits, batch["label"])
            if step == args.limit_val_batches:
                break
        val_acc = val_metric.compute().item()
        history["accuracy"].append(val_acc)
        tl = (total_loss / max(steps_per_epoch, 1)).item() if args.with_tracking else float("nan")
        history["train_loss_epoch"].append(tl)
        acc.print(f"epoch {epoch}: val accuracy {val_acc:.4f}  train clips/s {history['clips_per_sec'][-1]:.1f}")
        if args.with_tracking:
            acc.log({"accuracy": val_acc, "train_loss_epoch": tl, "epoch": epoch,
                     "clips_per_sec": history["clips_per_sec"][-1]}, step=epoch)
        if checkpointing_steps == "epoch":
            output_dir = os.path.join(args.output_dir or ".", f"epoch_{epoch}")
            acc.save_state(output_dir)

    bar.close()
    if args.with_tracking:
        acc.end_training()
    final_dir = output_dir or os.path.join(args.output_dir or ".", "final")
    acc.save_state(final_dir)
    history["final_dir"] = final_dir
    history["backend"] = backend.name
    history["global_step"] = global_step
    return history
