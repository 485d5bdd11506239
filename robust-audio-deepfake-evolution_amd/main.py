"""Train / eval CLI, drop-in for the reference's src/main.py on the MI355X path.

  python main.py --config config/Phase6_Proposed.conf [--output_dir ./exp_result] [--seed 1234]
                 [--eval] [--comment S] [--eval_model_weights P] [--resume P] [--start_epoch N]
                 [--pretrained_weights P] [--model ARCH]
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 main.py --config ...

Same flags, config keys and output layout as the reference (src/main.py:161-796, :1129-1175):
  {output_dir}/{track}_{confstem}_ep{E}_bs{B}[_{comment}]/
      config.conf, metric_log.txt, weights/epoch_{e}_{deer:.3f}.pth, weights/best.pth,
      weights/checkpoint_epoch_{e:03d}.pth (last 3 kept), weights/swa.pth,
      metrics/dev_score.txt, metrics/dev_t-DCF_EER_{e}epo.txt, metrics/t-DCF_EER_{e:03d}epo.txt,
      {eval_output}, t-DCF_EER.txt, eval_scores_2021DF.txt + t-DCF_EER_2021DF.txt (auto_eval_2021_df)
Extra flags: --amp {fp16,bf16,fp32} (default fp16: the reference's fp16 autocast + GradScaler, on the kernels of
libradhip_f16.so; bf16 runs the same kernels with bf16 storage, no GradScaler), --eager (no HIP graphs),
--loader-threads.

Differences, all documented in DESIGN.md:
  * data-parallel: one process per GPU (RCCL); the train list is sharded per global micro-step; by default
    an optimizer step keeps the reference's batch_size x accumulation_steps utterances, split over the ranks
    (radhip.train.ddp_micro_batches; --ddp_batch per_rank gives every rank the whole recipe), and eval
    shards the protocol and all-gathers the scores;
  * the train dataset is decoded natively and augmented on the GPU (radhip.data.TrainFeeder), with
    the reference's per-utterance host RNG order;
  * the optimizer window of `accumulation_steps` micro-batches runs as one batched clean pass plus the
    sequential FGM passes (radhip/window.py, same math; needs frozen BN) unless --no-window or --eager;
  * checkpoints load with torch.load(weights_only=True), strictly for --eval / --resume / auto 2021 DF
    (the reference's strict=False silently drops mismatched keys); tensorboard scalars are not written;
  * --save_train_state additionally writes weights/train_state_epoch_XXX.pt (last 2 kept) after every
    epoch: weights, optimizer, scheduler, scaler, EMA, SWA, best metrics, loader generator, host/device
    RNG states; --resume on such a file continues the run where it stopped.
"""
import argparse
import json
import math
import os
import random
import sys
from pathlib import Path
from shutil import copy

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")  # see radhip/__init__.py (graph memset replay)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from radhip.build import apply_lora_to_wavlm, get_model, load_weights  # noqa: E402
from radhip.data import (Dataset_ASVspoof2019_devNeval, Dataset_ASVspoof2021_eval, EvalFeeder,  # noqa: E402
                         TrainFeeder, genSpoof_list, str_to_bool)
from radhip.evaluation import calculate_EER_2021, calculate_tDCF_EER  # noqa: E402
from radhip.infer import produce_evaluation_file_sharded  # noqa: E402
from radhip.train import (Augmenter, GraphedMicroStep, Trainer, build_criterion,  # noqa: E402
                          ddp_micro_batches, swa_bn_update, total_optimizer_steps)
from radhip.window import WindowStep, window_eligible  # noqa: E402

AMP = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}
TRAIN_STATE_FORMAT = "radhip-train-state-v1"


def set_seed(seed, config):
    """src/utils.py:152-194: python, numpy, torch (+ device) seeds and the cudnn toggles."""
    if config is None:
        raise ValueError("config should not be None")
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
        torch.backends.cudnn.deterministic = str_to_bool(config["cudnn_deterministic_toggle"])
        torch.backends.cudnn.benchmark = str_to_bool(config["cudnn_benchmark_toggle"])


def model_tag_dir(args, config):
    tag = "{}_{}_ep{}_bs{}".format(config["track"], os.path.splitext(os.path.basename(args.config))[0],
                                   config["num_epochs"], config["batch_size"])
    if args.comment:
        tag += "_{}".format(args.comment)
    return Path(args.output_dir) / tag


def protocol_paths(config, track, database_path):
    p = "ASVspoof2019.{}".format(track)
    proto = database_path / "ASVspoof2019_{}_cm_protocols".format(track)
    trn = (Path(config["data_config"]["custom_train_protocol"])
           if "custom_train_protocol" in config.get("data_config", {}) else proto / "{}.cm.train.trn.txt".format(p))
    return trn, proto / "{}.cm.dev.trl.txt".format(p), proto / "{}.cm.eval.trl.txt".format(p)


class SWA:
    """torchcontrib SWA(optimizer).update_swa / swap_swa_sgd (src/main.py:488,644,672): running mean of
    the trainable tensors at every best-dev snapshot."""

    def __init__(self, params):
        self.params, self.buf, self.n = list(params), None, 0

    @torch.no_grad()
    def update(self):
        if self.buf is None:
            self.buf = [p.detach().clone() for p in self.params]
        else:
            for b, p in zip(self.buf, self.params):
                b.mul_(self.n / (self.n + 1)).add_(p.detach(), alpha=1.0 / (self.n + 1))
        self.n += 1

    @torch.no_grad()
    def swap(self):
        if self.buf is None:
            return
        for b, p in zip(self.buf, self.params):
            tmp = p.detach().clone()
            p.copy_(b)
            b.copy_(tmp)

    def state_dict(self):
        return {"n": self.n, "buf": None if self.buf is None else [b.detach().clone() for b in self.buf]}

    def load_state_dict(self, st):
        self.n = int(st["n"])
        self.buf = None if st["buf"] is None else [b.to(p.device) for b, p in zip(st["buf"], self.params)]


class Runner:
    def __init__(self, args):
        self.args = args
        with open(args.config) as f:
            config = json.loads(f.read())
        self.config = config
        self.model_config = config["model_config"]
        self.optim_config = config["optim_config"]
        self.optim_config["epochs"] = config["num_epochs"]
        self.track = config["track"]
        assert self.track in ["LA", "PA", "DF"], "Invalid track given"
        config.setdefault("eval_all_best", "True")
        config.setdefault("freq_aug", "False")
        self.tc = config.get("training_config", {})
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if not torch.cuda.is_available():
            raise RuntimeError("main.py runs the MI355X HIP path and needs a ROCm GPU (there is no CPU path)")
        torch.cuda.set_device(local)
        self.device = torch.device("cuda", local)
        if self.world > 1:
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            dist.init_process_group("nccl", device_id=self.device)
        set_seed(args.seed, config)
        self.database_path = Path(config["database_path"])
        self.tag = model_tag_dir(args, config)
        self.weights_dir = self.tag / "weights"
        self.eval_score_path = self.tag / config["eval_output"]
        if self.rank == 0:
            os.makedirs(self.weights_dir, exist_ok=True)
            copy(args.config, self.tag / "config.conf")
        self.amp = AMP[args.amp]
        self.threads = args.loader_threads

    def log(self, *a, **k):
        if self.rank == 0:
            print(*a, **k, flush=True)

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    # ------------------------------------------------------------------ model ------------------
    def build_model(self):
        args, mc = self.args, self.model_config
        mc["architecture"] = args.model if args.model else mc["architecture"]
        model = get_model(mc, self.device)
        self.log("no. model params:{}".format(sum(p.numel() for p in model.parameters())))
        model = apply_lora_to_wavlm(model, self.tc)
        if self.tc.get("freeze_sincnet", False) and hasattr(model, "sinc_stream"):
            for p in model.sinc_stream.parameters():
                p.requires_grad = False
        if args.pretrained_weights:
            self.log(f"Loading pretrained weights for fine-tuning: {args.pretrained_weights}")
            load_weights(model, args.pretrained_weights, self.device, strict=False)
        self.resume_state = None
        if args.resume:
            self.log("Resuming from checkpoint: {}".format(args.resume))
            ck = torch.load(args.resume, map_location=self.device, weights_only=True)
            if isinstance(ck, dict) and ck.get("format") == TRAIN_STATE_FORMAT:
                self.resume_state = ck      # full state: restored once the trainer exists (run())
            else:
                load_weights(model, args.resume, self.device, strict=True)
        return model

    # ------------------------------------------------------------------- eval ------------------
    def score(self, model, keys, base_dir, save_path, trial_path, fmt="2019", zero_on_error=False):
        ds_cls = Dataset_ASVspoof2021_eval if fmt == "2021" else Dataset_ASVspoof2019_devNeval
        ds = ds_cls(keys, base_dir)
        bs = int(self.config.get("test_config", {}).get("batch_size", self.config["batch_size"]))
        feeder = EvalFeeder(ds, bs, threads=self.threads, zero_on_error=zero_on_error)
        eval_amp = {"fp32": None, "x3": "x3"}.get(self.args.eval_amp) or AMP[self.args.eval_amp]
        produce_evaluation_file_sharded(ds, model, self.device, save_path, trial_path, batch_size=bs,
                                        criterion=self.criterion, batches=feeder.batches, fmt=fmt, amp=eval_amp)
        self.barrier()

    def tdcf(self, score_file, output_file, printout=True):
        """rank 0 computes, the (EER, t-DCF) pair is broadcast so every rank takes the same branch."""
        res = torch.zeros(2, dtype=torch.float64, device=self.device)
        if self.rank == 0:
            e, t = calculate_tDCF_EER(cm_scores_file=score_file,
                                      asv_score_file=self.database_path / self.config["asv_score_path"],
                                      output_file=output_file, printout=printout)
            res[0], res[1] = e, t
        if self.world > 1:
            dist.broadcast(res, 0)
        return float(res[0]), float(res[1])

    def run_eval(self, model):
        args, config = self.args, self.config
        model_path = args.eval_model_weights if args.eval_model_weights is not None else config["model_path"]
        load_weights(model, model_path, self.device, strict=True)
        self.log("Model loaded : {}".format(model_path))
        self.log("Start evaluation...")
        if config.get("is_eval_2021", False):
            trial = self.database_path / "ASVspoof2021.DF.cm.eval.trl.txt"
            keys = genSpoof_list(trial, is_train=False, is_eval=True, is_2021=True)
            self.log(f"no. evaluation files: {len(keys)}")
            self.score(model, keys, self.database_path, self.eval_score_path, trial, fmt="2021", zero_on_error=True)
            key_file = config.get("key_file", "./keys/DF/CM/trial_metadata.txt")
            if self.rank == 0:
                if Path(key_file).exists():
                    eer, _ = calculate_EER_2021(self.eval_score_path, key_file, self.tag / "t-DCF_EER_2021DF.txt")
                    print(f"ASVspoof 2021 DF EER: {eer:.4f}%")
                else:
                    print(f"Warning: Key file not found at {key_file}; scores saved but EER not computed.")
                print("DONE. Scores saved to: {}".format(self.eval_score_path))
            return
        _, _, eval_trial = protocol_paths(config, self.track, self.database_path)
        keys = genSpoof_list(eval_trial, is_train=False, is_eval=True)
        base = self.database_path / "ASVspoof2019_{}_eval/".format(self.track)
        self.score(model, keys, base, self.eval_score_path, eval_trial)
        self.tdcf(self.eval_score_path, self.tag / "t-DCF_EER.txt")
        self.log("DONE.")
        self.tdcf(self.eval_score_path, self.tag / "loaded_model_t-DCF_EER.txt")

    # ------------------------------------------------------------------ train ------------------
    def make_stepper(self, trainer, B):
        """How micro-batches execute: the accumulation window (HIP graphs, radhip/window.py), the
        per-micro-batch graphs (GraphedMicroStep), or eager launches."""
        if self.args.eager or not hasattr(trainer.model, "wavlm_stream"):
            return "eager", None        # the captured steps drive the dual-stream model's device-side draws
        # capture stages a dummy window (SpecAugment, LayerDrop and band-mask draws from numpy, torch CPU and
        # python random): put the host RNGs back afterwards, so a seeded run's first micro-batch draws what the
        # reference's first micro-batch draws
        rng = (random.getstate(), np.random.get_state(), torch.get_rng_state())
        try:
            if not self.args.no_window and window_eligible(trainer):
                w = WindowStep(trainer, B)
                for k in range(w.K):            # capture needs one staged window of draws
                    w.add(k, np.zeros(B, dtype=np.int64))
                w.capture()
                w.reset_host()
                return "window", w
            g = GraphedMicroStep(trainer, B)
            g.capture()
            return "graph", g
        finally:
            random.setstate(rng[0])
            np.random.set_state(rng[1])
            torch.set_rng_state(rng[2])

    def train_epoch(self, trainer, stepper, feeder, aug):
        """One pass of train_epoch (src/main.py:998-1126) over this rank's micro-batches."""
        kind, st = stepper
        trainer.begin_epoch()
        n_micro = len(feeder)
        K = st.K if kind == "window" else 1
        full = (n_micro // K) * K                  # micro-batches that fill whole windows
        for i, keys in enumerate(feeder.epoch()):
            flat, offs, lens, y = feeder.load(keys, self.device)
            plan = aug.draw(lens)
            lam, perm = trainer.mixup_draw(len(keys))
            last = i + 1 == n_micro
            if kind == "window" and i < full:
                k = i % K
                aug.run(flat, offs, lens, plan, perm, lam, out=st.xslot(k))
                st.add(k, y.numpy(), lam, perm)
                if k == K - 1:
                    st.run()
            elif kind == "graph":
                aug.run(flat, offs, lens, plan, perm, lam, out=st.x)
                st.run(y.numpy(), lam, perm, last_in_epoch=last)
            else:                                  # eager, or a trailing partial window
                x = aug.run(flat, offs, lens, plan, perm, lam)
                trainer.micro_step(x, y, lam, perm, last_in_epoch=last)

    def save_train_state(self, path, epoch, model, trainer, swa, feeder, best):
        """Full resume state (opt-in, --save_train_state): the reference keeps weights only."""
        nst = np.random.get_state()
        py = random.getstate()
        torch.save({"format": TRAIN_STATE_FORMAT, "epoch": epoch, "model": model.state_dict(),
                    "buffers": {n: b.detach().clone() for n, b in model.named_buffers()},
                    "trainer": trainer.state_dict(), "swa": swa.state_dict(), "best": dict(best),
                    "loader_gen": feeder.gen.get_state(),
                    "rng": {"python": [py[0], list(py[1]), py[2]],
                            "numpy": [nst[0], torch.from_numpy(nst[1].astype(np.int64)), int(nst[2]), int(nst[3]),
                                      float(nst[4])],
                            "torch": torch.get_rng_state(), "cuda": torch.cuda.get_rng_state(self.device)}},
                   path)

    def restore_train_state(self, st, model, trainer, swa, feeder, best):
        model.load_state_dict(st["model"], strict=True)
        with torch.no_grad():       # non-persistent buffers too (the encoder's device dropout seed), in place
            for n, b in model.named_buffers():
                b.copy_(st["buffers"][n])
        trainer.load_state_dict(st["trainer"])
        swa.load_state_dict(st["swa"])
        best.update(st["best"])
        r = st["rng"]
        random.setstate((r["python"][0], tuple(r["python"][1]), r["python"][2]))
        npk = r["numpy"]
        np.random.set_state((npk[0], npk[1].cpu().numpy().astype(np.uint32), npk[2], npk[3], npk[4]))
        torch.set_rng_state(r["torch"].cpu())          # (map_location put every tensor on the device)
        torch.cuda.set_rng_state(r["cuda"].cpu(), self.device)
        feeder.gen.set_state(st["loader_gen"].cpu())
        return int(st["epoch"]) + 1

    def run(self):
        args, config = self.args, self.config
        model = self.build_model()
        self.criterion = build_criterion(config, self.device)
        if args.eval:
            self.run_eval(model)
            return
        trn_list, dev_trial, eval_trial = protocol_paths(config, self.track, self.database_path)
        d_label_trn, file_train = genSpoof_list(trn_list, is_train=True, is_eval=False)
        self.log("no. training files:", len(file_train))
        dc = config.get("data_config", {})
        aug = Augmenter(self.device, algo=int(dc.get("rawboost_algo", 0)), rawboost_p=float(dc.get("rawboost_p", 1.0)),
                        use_codec=str_to_bool(dc.get("use_codec_aug", "False")), codec_p=float(dc.get("codec_p", 0.5)),
                        exact_noise=args.exact_rawboost)
        B = int(config["batch_size"])
        if self.world > 1 and args.ddp_batch == "global":
            # the reference's optimizer step (batch_size x accumulation_steps utterances) split over the ranks
            glob = B * max(1, int(self.tc.get("accumulation_steps", 1)))
            B, acc = ddp_micro_batches(B, self.tc.get("accumulation_steps", 1), self.world)
            self.tc["accumulation_steps"] = acc
            self.log(f"[DDP] global batch {glob} per optimizer step: per-rank micro-batch {B} x accumulation {acc} "
                     f"x {self.world} ranks")
        feeder = TrainFeeder(file_train, d_label_trn, self.database_path / "ASVspoof2019_{}_train/".format(self.track),
                             B, aug, args.seed, threads=self.threads, rank=self.rank, world=self.world)
        if len(feeder) == 0:
            raise RuntimeError(f"{len(file_train)} training files are fewer than one global batch "
                               f"({self.world} x {B})")
        _, file_dev = genSpoof_list(dev_trial, is_train=False, is_eval=False)
        file_eval = genSpoof_list(eval_trial, is_train=False, is_eval=True)
        self.log("no. validation files:", len(file_dev))
        dev_base = self.database_path / "ASVspoof2019_{}_dev/".format(self.track)
        eval_base = self.database_path / "ASVspoof2019_{}_eval/".format(self.track)

        accum = max(1, int(self.tc.get("accumulation_steps", 1)))
        steps_per_epoch = math.ceil(len(feeder) / accum)
        total = config["num_epochs"] * steps_per_epoch
        trainer = Trainer(model, config, self.device, total, self.amp, world_group=None, criterion=self.criterion)
        self.log(f"[Schedule] micro-batches/epoch={len(feeder)}, accumulation_steps={accum} -> "
                 f"optimizer_steps/epoch={steps_per_epoch}, total_steps={total}")
        swa = SWA(trainer.params)
        best = {"dev_eer": 100.0, "eval_eer": 100.0, "dev_tdcf": 100.0, "eval_tdcf": 100.0}
        start = args.start_epoch
        # graph capture consumes host RNG draws and runs warm-up passes, so it happens before a full
        # resume restores the RNG / device-seed / optimizer state of the interrupted run
        stepper = self.make_stepper(trainer, B)
        self.log(f"[Step] micro-batches execute as: {stepper[0]}")
        if self.resume_state is not None:
            start = self.restore_train_state(self.resume_state, model, trainer, swa, feeder, best)
            self.log(f"Resumed the full training state; continuing at epoch {start}")
            self.resume_state = None
        metric_path = self.tag / "metrics"
        if self.rank == 0:
            os.makedirs(metric_path, exist_ok=True)
            with open(self.tag / "metric_log.txt", "a") as f_log:
                f_log.write("=" * 5 + "\n")
        for epoch in range(start, config["num_epochs"]):
            self.log("Start training epoch{:03d}".format(epoch))
            self.train_epoch(trainer, stepper, feeder, aug)
            running_loss = trainer.epoch_loss()
            # dev / eval scoring and best-model files with the EMA weights when enabled (the reference's
            # eval_model = ema_model); SWA averages the live optimizer parameters afterwards
            if trainer.ema is not None:
                trainer.ema.swap()
            self.score(model, file_dev, dev_base, metric_path / "dev_score.txt", dev_trial)
            dev_eer, dev_tdcf = self.tdcf(metric_path / "dev_score.txt",
                                          metric_path / "dev_t-DCF_EER_{}epo.txt".format(epoch), printout=False)
            self.log("DONE.\nLoss:{:.5f}, dev_eer: {:.3f}, dev_tdcf:{:.5f}".format(running_loss, dev_eer, dev_tdcf))
            best["dev_tdcf"] = min(dev_tdcf, best["dev_tdcf"])
            improved = best["dev_eer"] >= dev_eer
            if improved:
                self.log("best model find at epoch", epoch)
                best["dev_eer"] = dev_eer
                name = "epoch_{}_{:03.3f}.pth".format(epoch, dev_eer)
                if self.rank == 0:
                    for old in self.weights_dir.glob("epoch_*_*.pth"):
                        if old.name != name:
                            old.unlink(missing_ok=True)
                    torch.save(model.state_dict(), self.weights_dir / name)
                if str_to_bool(config["eval_all_best"]):
                    self.score(model, file_eval, eval_base, self.eval_score_path, eval_trial)
                    eval_eer, eval_tdcf = self.tdcf(self.eval_score_path,
                                                    metric_path / "t-DCF_EER_{:03d}epo.txt".format(epoch))
                    log_text = "epoch{:03d}, ".format(epoch)
                    if eval_eer < best["eval_eer"]:
                        log_text += "best eer, {:.4f}%".format(eval_eer)
                        best["eval_eer"] = eval_eer
                    if eval_tdcf < best["eval_tdcf"]:
                        log_text += "best tdcf, {:.4f}".format(eval_tdcf)
                        best["eval_tdcf"] = eval_tdcf
                        if self.rank == 0:
                            torch.save(model.state_dict(), self.weights_dir / "best.pth")
                    self.log(log_text)
                    if self.rank == 0:
                        with open(self.tag / "metric_log.txt", "a") as f_log:
                            f_log.write(log_text + "\n")
            if trainer.ema is not None:
                trainer.ema.swap()
            if improved:
                self.log("Saving epoch {} for swa".format(epoch))
                swa.update()
            if ((epoch + 1) % 10 == 0 or epoch == config["num_epochs"] - 1) and self.rank == 0:
                ck = self.weights_dir / "checkpoint_epoch_{:03d}.pth".format(epoch)
                torch.save(model.state_dict(), ck)
                cks = sorted(self.weights_dir.glob("checkpoint_epoch_*.pth"), key=lambda x: int(x.stem.split("_")[-1]))
                for old in cks[:-3]:
                    old.unlink(missing_ok=True)
            if args.save_train_state and self.rank == 0:
                self.save_train_state(self.weights_dir / "train_state_epoch_{:03d}.pt".format(epoch), epoch, model,
                                      trainer, swa, feeder, best)
                sts = sorted(self.weights_dir.glob("train_state_epoch_*.pt"), key=lambda x: int(x.stem.split("_")[-1]))
                for old in sts[:-2]:
                    old.unlink(missing_ok=True)
        self.log("Start final evaluation")
        # reference order (src/main.py:669-690): swap the SWA average into the live model, bn_update over
        # the train loader, evaluate the EMA model if enabled (its own weights and construction-time
        # buffers, which bn_update does not touch) else the live model, save swa.pth = live model.
        final_state = None
        if trainer.ema is not None:
            trainer.ema.swap()
            self.score(model, file_eval, eval_base, self.eval_score_path, eval_trial)
            eval_eer, eval_tdcf = self.tdcf(self.eval_score_path, self.tag / "t-DCF_EER.txt")
            final_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
            trainer.ema.swap()
        if swa.n > 0:
            swa.swap()
            n_bn = swa_bn_update(model, feeder, aug, self.device)
            self.log(f"[SWA] averaged {swa.n} snapshots; BatchNorm statistics recomputed over {n_bn} utterances")
        if trainer.ema is None:
            self.score(model, file_eval, eval_base, self.eval_score_path, eval_trial)
            eval_eer, eval_tdcf = self.tdcf(self.eval_score_path, self.tag / "t-DCF_EER.txt")
            final_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
        if self.rank == 0:
            with open(self.tag / "metric_log.txt", "a") as f_log:
                f_log.write("=" * 5 + "\n")
                f_log.write("EER: {:.3f}, min t-DCF: {:.5f}".format(eval_eer, eval_tdcf))
            torch.save(model.state_dict(), self.weights_dir / "swa.pth")
        if eval_eer <= best["eval_eer"]:
            best["eval_eer"] = eval_eer
        if eval_tdcf <= best["eval_tdcf"]:
            best["eval_tdcf"] = eval_tdcf
            if self.rank == 0:
                torch.save(final_state, self.weights_dir / "best.pth")
        self.log("Exp FIN. EER: {:.3f}, min t-DCF: {:.5f}".format(best["eval_eer"], best["eval_tdcf"]))
        if config.get("auto_eval_2021_df", False):
            self.auto_eval_2021(model)
        if self.world > 1:
            dist.destroy_process_group()

    def auto_eval_2021(self, model):
        """src/main.py:698-796: score the 2021 DF set with best.pth (or the newest epoch model)."""
        config = self.config
        root = config.get("database_path_2021")
        key_file = config.get("key_file_2021", "/root/aasist-main/keys/DF/CM/trial_metadata.txt")
        if root is None:
            self.log("Warning: database_path_2021 not configured; skipping 2021 DF evaluation.")
            return
        trial = Path(root) / "ASVspoof2021.DF.cm.eval.trl.txt"
        if not trial.exists():
            self.log(f"Error: Protocol file not found: {trial}")
            return
        best = self.weights_dir / "best.pth"
        if not best.exists():
            eps = sorted(self.weights_dir.glob("epoch_*_*.pth"), key=lambda x: x.stat().st_mtime)
            if not eps:
                self.log("Error: No model found for 2021 evaluation.")
                return
            best = eps[-1]
        load_weights(model, best, self.device, strict=True)
        keys = genSpoof_list(trial, is_train=False, is_eval=True, is_2021=True)
        out = self.tag / "eval_scores_2021DF.txt"
        self.score(model, keys, Path(root), out, trial, fmt="2021", zero_on_error=True)
        if self.rank == 0:
            if Path(key_file).exists():
                eer, _ = calculate_EER_2021(out, key_file, self.tag / "t-DCF_EER_2021DF.txt")
                with open(self.tag / "metric_log.txt", "a") as f_log:
                    f_log.write("\n" + "=" * 5 + "\nASVspoof 2021 DF Evaluation (Cross-domain):\n")
                    f_log.write("EER: {:.4f}%\n".format(eer))
            else:
                print(f"Warning: Key file not found: {key_file}; scores saved to {out}")


def parse_args(argv=None):
    parser = argparse.ArgumentParser(description="ASVspoof detection system (MI355X path)")
    parser.add_argument("--config", dest="config", type=str, help="configuration file", required=True)
    parser.add_argument("--output_dir", dest="output_dir", type=str, help="output directory for results",
                        default="./exp_result")
    parser.add_argument("--seed", type=int, default=1234, help="random seed (default: 1234)")
    parser.add_argument("--eval", action="store_true", help="when this flag is given, evaluates given model and exit")
    parser.add_argument("--comment", type=str, default=None, help="comment to describe the saved model")
    parser.add_argument("--eval_model_weights", type=str, default=None, help="directory to the model weight file")
    parser.add_argument("--resume", type=str, default=None, help="path to checkpoint to resume from")
    parser.add_argument("--start_epoch", type=int, default=0, help="epoch to start training from")
    parser.add_argument("--pretrained_weights", type=str, default=None, help="pretrained weights for fine-tuning")
    parser.add_argument("--model", type=str, default=None, help="override the model architecture")
    parser.add_argument("--amp", default="fp16", choices=sorted(AMP), help="autocast dtype (reference: fp16)")
    parser.add_argument("--eval_amp", default="x3", choices=["x3", "fp32", "bf16", "fp16"],
                        help="scoring precision: x3 (default), the reference's fp32 scoring (src/main.py:958-995, no "
                             "autocast) with the WavLM stream on the hand-written split-precision kernels "
                             "(radhip/wavlm_x3.py: bf16 hi/lo planes, three MFMA products per GEMM, fp32 attention; "
                             "scores within 2e-6 of fp32, 2.2x its rate: tools/bench_eval.py); fp32, the same forward "
                             "with the WavLM stream on torch SDPA + hipBLASLt fp32; or bf16 / fp16 autocast, which "
                             "runs the hand-written HIP encoder / SincNet path (tools/bench_eval.py: throughput and "
                             "score deviation). 16-bit scores are parity-unpinned against the reference (no fixture "
                             "pins its EER); with --eval_amp bf16 / fp16 they also drive the dev-set best-model "
                             "selection")
    parser.add_argument("--eager", action="store_true", help="launch kernel by kernel (no HIP graphs)")
    parser.add_argument("--no-window", dest="no_window", action="store_true",
                        help="replay one graph pair per micro-batch instead of the batched accumulation window")
    parser.add_argument("--save_train_state", action="store_true",
                        help="also write weights/train_state_epoch_XXX.pt (optimizer, scheduler, EMA, SWA, RNG) for an "
                             "exact --resume")
    parser.add_argument("--loader-threads", dest="loader_threads", type=int, default=8,
                        help="host threads of the native FLAC batch decoder")
    parser.add_argument("--ddp_batch", default="global", choices=["global", "per_rank"],
                        help="data parallel: 'global' keeps the reference's batch_size x accumulation_steps utterances "
                             "per optimizer step split over the ranks (default); 'per_rank' gives every rank "
                             "batch_size x accumulation_steps (weak scaling, as bench.py)")
    parser.add_argument("--exact_rawboost", action="store_true",
                        help="draw the RawBoost ISD / SSI noise with the reference's numpy calls (randn / choice per "
                             "sample) instead of one Philox seed per call")
    return parser.parse_args(argv)


def main(args):
    Runner(args).run()


if __name__ == "__main__":
    main(parse_args())
