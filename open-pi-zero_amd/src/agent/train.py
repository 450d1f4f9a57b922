"""TrainAgent: the reference's training loop (train.py:36-560) on the native MI355X path.

Same structure and semantics as shroglck/open-pi-zero's TrainAgent:
  * one process per GPU (torchrun), ``PiZero(cfg, use_ddp)``, tie + freeze,
    bf16 weights, data-parallel wrapper with ``no_sync`` for accumulation;
  * two optimizers (action expert / VLM) with CosineAnnealingWarmupRestarts,
    joint grad-norm clip, ``zero_grad(set_to_none=True)``;
  * flow-matching time sampling (beta / uniform), per-batch preprocessing into
    the 9 forward kwargs (pizero.py:607-618);
  * checkpoints with the reference's keys (cnt_update, cnt_batch, model,
    action_optimizer, vlm_optimizer, *_lr_scheduler, wandb_id, n_averaged).
MI355X-native pieces: pizero_native.ddp.PiZeroDDP (RCCL bucketed all-reduce
overlapped with backward), pizero_native.optim.FusedAdamW (flat fused AdamW; by default
with the reference's blockwise 8-bit state, ``optimizer_state_bits: 8`` -- the algorithm of
bitsandbytes' AdamW8bit restated, bitsandbytes itself absent: parity with it unpinned).
Data: the OXE/RLDS TensorFlow pipeline is out of scope; the
agent consumes any iterable of reference-format batches, by default
``SyntheticBridgeDataset`` (bridge-shaped random batches, already tokenized).
"""

from __future__ import annotations

import logging
import os
from collections import deque

import numpy as np
import torch

from src.utils.config import cfg_get

log = logging.getLogger(__name__)


def sample_fm_time(bsz, flow_sampling="beta", beta_dist=None, t_max=1 - 0.001):
    """train.py:239-247: beta -> t = t_max * (1 - Beta(alpha, beta)); uniform -> stratified
    (U + arange(B)/B) mod (1 - 1e-5).  Same torch RNG calls as the reference (seeded parity)."""
    if flow_sampling == "uniform":
        return (torch.rand(1) + torch.arange(bsz) / bsz) % (1 - 1e-5)
    if flow_sampling != "beta":
        raise ValueError(f"Invalid flow matching timestep sampling mode: {flow_sampling}")
    return t_max * (1 - beta_dist.sample((bsz,)))


class SyntheticBridgeDataset(torch.utils.data.IterableDataset):
    """Reference batch format (train.py:319-327) with tokenized text (no tokenizer offline)."""

    def __init__(self, cfg, batch_size, seed=0):
        self.cfg, self.B, self.seed = cfg, batch_size, seed

    def __iter__(self):
        g = torch.Generator().manual_seed(self.seed)
        c = self.cfg
        P = cfg_get(c, "max_seq_len")
        n_img = cfg_get(c, "vision.config.num_image_tokens")
        H = cfg_get(c, "horizon_steps")
        img = cfg_get(c, "vision.config.image_size")
        vmax = min(int(cfg_get(c, "vocab_size")), int(cfg_get(c, "image_token_index")))
        nl = min(108, vmax - 1)
        while True:
            ids = torch.zeros(self.B, P, dtype=torch.int64)
            ids[:, :n_img] = cfg_get(c, "image_token_index")
            ids[:, n_img] = 2
            for b in range(self.B):
                n = int(torch.randint(4, P - n_img, (1,), generator=g))
                ids[b, n_img + 1 : n_img + n - 1] = torch.randint(3, vmax, (n - 2,), generator=g)
                ids[b, n_img + n - 1] = nl
            yield {
                "input_ids": ids,
                "attention_mask": (ids != 0).long(),
                "pixel_values": torch.randint(0, 256, (self.B, 3, img, img), generator=g, dtype=torch.uint8),
                "proprio": torch.rand(self.B, cfg_get(c, "cond_steps"), cfg_get(c, "proprio_dim"), generator=g) * 2 - 1,
                "action": torch.rand(self.B, H, cfg_get(c, "action_dim"), generator=g) * 2 - 1,
            }


class TrainAgent:
    def __init__(self, cfg, dataset=None):
        from pizero_native.ddp import PiZeroDDP
        from pizero_native.optim import FusedAdamW
        from src.model.vla.pizero import PiZero
        from src.utils.optim import CosineAnnealingWarmupRestarts

        self.cfg = cfg
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.multi_gpu = self.world > 1
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", cfg_get(cfg, "gpu_id", 0)))
        self.device = torch.device(f"cuda:{self.local_rank}")
        torch.cuda.set_device(self.device)
        if self.multi_gpu and not torch.distributed.is_initialized():
            torch.distributed.init_process_group("nccl", device_id=self.device)
        self.main_rank = self.rank == 0
        self.dtype = torch.bfloat16 if cfg_get(cfg, "use_bf16", True) else torch.float32
        self.n_updates = int(cfg_get(cfg, "n_updates", 1))
        self.max_grad_norm = float(cfg_get(cfg, "max_grad_norm", 1.0))
        self.log_freq = int(cfg_get(cfg, "log_freq", 16))
        self.save_model_freq = int(cfg_get(cfg, "save_model_freq", 10 ** 9))
        self.log_dir = cfg_get(cfg, "log_dir", "") or "."
        self.checkpoint_dir = os.path.join(self.log_dir, "checkpoint")

        self.cnt_update = 0
        self.cnt_batch = 0
        self.wandb_id = None
        model = PiZero(cfg, use_ddp=self.multi_gpu, device=self.device, dtype=self.dtype, init="default")
        self.model = model
        resume = cfg_get(cfg, "resume_checkpoint_path")
        if resume:
            self.load_checkpoint(resume)
        elif cfg_get(cfg, "load_pretrained_weights", False):
            model.load_pretrained_weights()
        model.tie_action_proprio_weights()
        model.freeze_unused_weights()
        self.model_meta = PiZeroDDP(model) if self.multi_gpu else model

        per_dev = int(cfg_get(cfg, "per_device_batch_size"))
        self.grad_accumulation_steps = max(int(cfg_get(cfg, "global_batch_size")) // per_dev // self.world, 1)
        self.train_dataloader = dataset if dataset is not None else SyntheticBridgeDataset(cfg, per_dev, seed=self.rank)

        self.train_vlm = bool(cfg_get(cfg, "train_vlm", True))
        # the reference's bnb AdamW8bit (train.py:171-175): blockwise 8-bit state by default
        self.state_bits = int(cfg_get(cfg, "optimizer_state_bits", 8))
        self.action_optimizer = FusedAdamW(model.action_expert_parameters, lr=cfg_get(cfg, "action_lr"),
                                           weight_decay=cfg_get(cfg, "action_weight_decay", 0.0),
                                           state_bits=self.state_bits)
        sch = lambda opt, key, lr: CosineAnnealingWarmupRestarts(  # noqa: E731
            opt, first_cycle_steps=cfg_get(cfg, f"{key}.first_cycle_steps"), cycle_mult=1.0, max_lr=lr,
            min_lr=cfg_get(cfg, f"{key}.min_lr"), warmup_steps=cfg_get(cfg, f"{key}.warmup_steps"), gamma=1.0)
        self.action_lr_scheduler = sch(self.action_optimizer, "action_lr_scheduler", cfg_get(cfg, "action_lr"))
        self.optimizers = [self.action_optimizer]
        if self.train_vlm:
            self.vlm_optimizer = FusedAdamW(model.trainable_vlm_parameters, lr=cfg_get(cfg, "vlm_lr"),
                                            weight_decay=cfg_get(cfg, "vlm_weight_decay", 0.0),
                                            state_bits=self.state_bits)
            self.vlm_lr_scheduler = sch(self.vlm_optimizer, "vlm_lr_scheduler", cfg_get(cfg, "vlm_lr"))
            self.optimizers.append(self.vlm_optimizer)
        else:
            for p in model.trainable_vlm_parameters:
                p.requires_grad = False
        self.flow_sampling = cfg_get(cfg, "flow_sampling", "beta")
        self.flow_t_max = 1 - float(cfg_get(cfg, "flow_sig_min", 0.001))
        self.flow_beta_dist = torch.distributions.Beta(float(cfg_get(cfg, "flow_alpha", 1.5)),
                                                       float(cfg_get(cfg, "flow_beta", 1)))
        if resume:
            self.load_optimizer(resume)

    def sample_fm_time(self, bsz):
        """train.py:239-247."""
        return sample_fm_time(bsz, self.flow_sampling, self.flow_beta_dist, self.flow_t_max)

    def preprocess_batch(self, batch, split_mask=False, sample_fm_time=True):
        """train.py:271-314 with the per-batch work on the device: the raw batch
        (int64 ids / attention mask, uint8 pixels, fp32 proprio / actions) is copied once, then the
        block mask + positions (vectorised builder, pizero.py:271-324) and the pixel normalisation
        (x/255 - 0.5)/0.5 (vla/processing.py:109-114) are computed on the GPU -- no per-sample host
        loop, and 1 byte per pixel crosses PCIe instead of 2."""
        m = self.model
        dev = self.device
        nb = dict(non_blocking=True)
        am = batch["attention_mask"].to(dev, **nb)
        mask, vpos, ppos, apos = m.build_causal_mask_and_position_ids(am, self.dtype)
        pix = batch["pixel_values"].to(dev, **nb)
        if pix.dtype == torch.uint8:
            pix = (pix.to(torch.float32) / 255.0 - 0.5) / 0.5
        inputs = {"input_ids": batch["input_ids"].to(dev, **nb), "pixel_values": pix.to(self.dtype),
                  "vlm_position_ids": vpos, "proprio_position_ids": ppos, "action_position_ids": apos,
                  "proprios": batch["proprio"].to(dev, **nb).to(self.dtype),
                  "actions": batch["action"].to(dev, **nb).to(self.dtype)}
        if split_mask:
            inputs["image_text_proprio_mask"], inputs["action_mask"] = m.split_full_mask_into_submasks(mask)
        else:
            inputs["causal_mask"] = mask
        if sample_fm_time:
            inputs["t"] = self.sample_fm_time(len(batch["input_ids"])).to(dev, **nb).to(self.dtype)
        return inputs

    def run(self):
        from pizero_native.optim import clip_grad_norm_

        loss_deque = deque(maxlen=self.grad_accumulation_steps)
        self.model_meta.train()
        it = iter(self.train_dataloader)
        while self.cnt_update < self.n_updates:
            batch = next(it)
            inputs = self.preprocess_batch(batch)
            last = (self.cnt_batch + 1) % self.grad_accumulation_steps == 0
            ctx = self.model_meta.no_sync() if (self.multi_gpu and not last) else torch.enable_grad()
            with ctx:
                loss = self.model_meta(**inputs)
                (loss / self.grad_accumulation_steps).backward()
            if last:
                clip_grad_norm_(self.optimizers, self.max_grad_norm)
                for opt in self.optimizers:
                    opt.step()
                self.action_lr_scheduler.step()
                if self.train_vlm:
                    self.vlm_lr_scheduler.step()
                for opt in self.optimizers:
                    opt.zero_grad(set_to_none=True)
                self.cnt_update += 1
                if self.cnt_update % self.save_model_freq == 0 or self.cnt_update == self.n_updates:
                    self.save_training(self.cnt_update, self.cnt_batch)
            # every micro-batch's loss enters the window (kept on the device: no sync), as the reference's
            # deque of grad_accumulation_steps rank-mean losses (train.py:405-463); the window is all-reduced
            # ONCE, on the logged batches only (every rank has the same cnt_batch, so all enter the collective)
            loss_deque.append(loss.detach().reshape(1).float())
            if self.cnt_batch % self.log_freq == 0:
                win = torch.cat(list(loss_deque))
                if self.multi_gpu:
                    torch.distributed.all_reduce(win, op=torch.distributed.ReduceOp.SUM)
                    win = win / self.world
                if self.main_rank:
                    log.info("Batch %d Update %d: loss %.4f | action lr %.8f", self.cnt_batch, self.cnt_update,
                             float(win.mean()), self.action_optimizer.param_groups[0]["lr"])
            self.cnt_batch += 1
        return self

    # ---------------------------------------------------------- checkpoints --
    def save_training(self, cnt_update, cnt_batch):
        if not self.main_rank or not cfg_get(self.cfg, "log_dir"):
            return None
        os.makedirs(self.checkpoint_dir, exist_ok=True)
        data = {
            "cnt_update": cnt_update, "cnt_batch": cnt_batch,
            "model": {k: v.detach().clone() for k, v in self.model.state_dict().items()},
            "action_optimizer": self.action_optimizer.state_dict(),
            "vlm_optimizer": self.vlm_optimizer.state_dict() if self.train_vlm else None,
            "action_lr_scheduler": self.action_lr_scheduler.state_dict(),
            "vlm_lr_scheduler": self.vlm_lr_scheduler.state_dict() if self.train_vlm else None,
            "wandb_id": None, "n_averaged": 1,
        }
        path = os.path.join(self.checkpoint_dir, f"step{cnt_update}.pt")
        torch.save(data, path)
        return path

    def load_checkpoint(self, path):
        """train.py:531-544: counters + weights (strict, ``_orig_mod.`` prefix of compiled saves stripped)."""
        data = torch.load(path, weights_only=True, map_location="cpu")
        self.cnt_update = int(data["cnt_update"])
        self.cnt_batch = int(data["cnt_batch"])
        self.wandb_id = data.get("wandb_id")
        sd = {k.replace("_orig_mod.", ""): v for k, v in data["model"].items()}
        self.model.load_state_dict(sd, strict=True)
        log.info("Loaded model from %s at update %d batch %d", path, self.cnt_update, self.cnt_batch)
        return data

    def load_optimizer(self, path):
        """train.py:546-560: optimizer moments/steps and scheduler states."""
        data = torch.load(path, weights_only=True, map_location="cpu")
        self.action_optimizer.load_state_dict(data["action_optimizer"])
        self.action_lr_scheduler.load_state_dict(data["action_lr_scheduler"])
        if self.train_vlm:
            self.vlm_optimizer.load_state_dict(data["vlm_optimizer"])
            self.vlm_lr_scheduler.load_state_dict(data["vlm_lr_scheduler"])
        log.info("Loaded optimizer and scheduler states from %s", path)
