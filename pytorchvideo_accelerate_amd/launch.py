"""``accelerate launch`` equivalent for this engine (SURVEY.md D1, §5 failure detection).

    python -m pytorchvideo_accelerate_amd.launch [--config_file cfg.yaml] [--multi_gpu] [--num_processes N]
        [--cpu] [--mixed_precision bf16] [--max_restarts R] [--auto_resume] run.py --is_slowfast ...

* Reads the accelerate YAML config (``--config_file``, else ``$ACCELERATE_CONFIG_FILE``, else
  ``$HF_HOME/accelerate/default_config.yaml`` / ``~/.cache/huggingface/accelerate/default_config.yaml``) with
  ``yaml.safe_load``; command-line flags override it (accelerate precedence).
* With no config file, an unset ``--num_processes`` becomes the number of visible GPUs, and more than one GPU turns
  on multi-GPU training (accelerate's defaults, ``[acc] commands/launch.py:1302-1340``), so the reference's bare
  ``accelerate launch run.py ...`` (``run_slowfast_r50.sh:1``) starts one rank per GPU.  The count comes from
  ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` when set, else from a throwaway child
  process, so the launcher itself never initialises the GPU.
* One process on one machine: the script runs as a child process (accelerate's ``simple_launcher``).
  Otherwise ``python -m torch.distributed.run`` (elastic agent) starts ``num_processes // num_machines``
  ranks per node — one process per GPU, RCCL over xGMI — with ``--max_restarts``/``--monitor_interval``.
* Environment contract for the script: ``ACCELERATE_MIXED_PRECISION``, ``ACCELERATE_USE_CPU``, and
  ``PVA_AUTO_RESUME=1`` with ``--auto_resume`` (the trainer then resumes from the newest ``step_*``/``epoch_*``
  checkpoint after an elastic restart).  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is kept for RCCL on this host.
* The launcher never replaces itself (no ``exec``): it waits for the child and exits with its code.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from typing import Dict, List, Optional, Tuple

DEFAULTS = {"distributed_type": "NO", "num_processes": None, "num_machines": 1, "machine_rank": 0,
            "main_process_ip": "127.0.0.1", "main_process_port": 29500, "mixed_precision": "no", "use_cpu": False,
            "gpu_ids": "all", "max_restarts": 0, "monitor_interval": 5.0, "rdzv_backend": "static"}


def default_config_path() -> str:
    if os.environ.get("ACCELERATE_CONFIG_FILE"):
        return os.environ["ACCELERATE_CONFIG_FILE"]
    hf = os.environ.get("HF_HOME", os.path.join(os.path.expanduser("~"), ".cache", "huggingface"))
    return os.path.join(hf, "accelerate", "default_config.yaml")


def _visible_from_env() -> Optional[int]:
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(k)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() not in ("", "-1")])
    return None


def _device_count() -> int:
    """Visible GPUs without initialising a GPU in this process (env masks, else ``torch.cuda.device_count()`` in a
    throwaway child; 0 when that fails)."""
    n = _visible_from_env()
    if n is not None:
        return n
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=300)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else 0
    except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
        return 0


def load_config(path: Optional[str]) -> Dict:
    """accelerate config file (YAML or JSON) -> dict of the keys this launcher understands (``from_file``: whether
    a config file was found)."""
    cfg = dict(DEFAULTS)
    cfg["from_file"] = False
    p = path or default_config_path()
    if p and os.path.exists(p):
        cfg["from_file"] = True
        import yaml
        with open(p) as f:
            raw = yaml.safe_load(f) or {}
        for k in DEFAULTS:
            if k in raw and raw[k] is not None:
                cfg[k] = raw[k]
    elif path:
        raise FileNotFoundError(f"accelerate config file not found: {path}")
    return cfg


def parse(argv: List[str]) -> Tuple[argparse.Namespace, List[str]]:
    ap = argparse.ArgumentParser(prog="pytorchvideo_accelerate_amd.launch", allow_abbrev=False)
    ap.add_argument("--config_file", default=None)
    ap.add_argument("--cpu", action="store_true", default=None)
    ap.add_argument("--multi_gpu", action="store_true")
    ap.add_argument("--num_processes", type=int, default=None)
    ap.add_argument("--num_machines", type=int, default=None)
    ap.add_argument("--machine_rank", type=int, default=None)
    ap.add_argument("--main_process_ip", default=None)
    ap.add_argument("--main_process_port", type=int, default=None)
    ap.add_argument("--mixed_precision", choices=["no", "fp16", "bf16"], default=None)
    ap.add_argument("--gpu_ids", default=None)
    ap.add_argument("--max_restarts", type=int, default=None)
    ap.add_argument("--monitor_interval", type=float, default=None)
    ap.add_argument("--rdzv_backend", default=None)
    ap.add_argument("--auto_resume", action="store_true", help="resume from the newest checkpoint after a restart")
    ap.add_argument("-m", "--module", action="store_true", help="the script is a python module")
    ap.add_argument("training_script")
    ap.add_argument("training_script_args", nargs=argparse.REMAINDER)
    return ap.parse_known_args(argv)[0], []


def resolve(a: argparse.Namespace) -> Dict:
    cfg = load_config(a.config_file)
    for k in ("num_processes", "num_machines", "machine_rank", "main_process_ip", "main_process_port",
              "mixed_precision", "gpu_ids", "max_restarts", "monitor_interval", "rdzv_backend"):
        v = getattr(a, k)
        if v is not None:
            cfg[k] = v
    if a.cpu is not None:
        cfg["use_cpu"] = a.cpu
    if cfg["num_processes"] is None:
        if cfg["from_file"] or cfg["use_cpu"]:
            cfg["num_processes"] = 1
        else:
            # accelerate without a config: one rank per visible GPU (warned, as accelerate does)
            n = _device_count()
            cfg["num_processes"] = max(n, 1)
            print(f"[launch] `--num_processes` was set to a value of `{cfg['num_processes']}`", file=sys.stderr)
            if n > 1 and not a.multi_gpu:
                print("[launch] More than one GPU was found, enabling multi-GPU training. If this was unintended "
                      "please pass in `--num_processes=1`.", file=sys.stderr)
                a.multi_gpu = True
    if a.multi_gpu:
        cfg["distributed_type"] = "MULTI_GPU"
    if cfg["use_cpu"] and int(cfg["num_processes"]) > 1:
        cfg["distributed_type"] = "MULTI_CPU"
    return cfg


def build_command(a: argparse.Namespace, cfg: Dict) -> Tuple[List[str], Dict[str, str]]:
    env = dict(os.environ)
    env["ACCELERATE_MIXED_PRECISION"] = str(cfg["mixed_precision"])
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if cfg["use_cpu"]:
        env["ACCELERATE_USE_CPU"] = "true"
    if a.auto_resume:
        env["PVA_AUTO_RESUME"] = "1"
    if str(cfg["gpu_ids"]) not in ("all", "None", ""):
        env["HIP_VISIBLE_DEVICES"] = str(cfg["gpu_ids"])
    target = (["-m", a.training_script] if a.module else [a.training_script]) + list(a.training_script_args)
    nproc, nnodes = int(cfg["num_processes"]), int(cfg["num_machines"])
    if nproc <= 1 and nnodes <= 1 and int(cfg["max_restarts"]) == 0:
        return [sys.executable] + target, env
    per_node = max(1, nproc // max(nnodes, 1))
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nnodes={nnodes}", f"--nproc-per-node={per_node}",
           f"--max-restarts={cfg['max_restarts']}", f"--monitor-interval={cfg['monitor_interval']}"]
    endpoint = f"{cfg['main_process_ip']}:{cfg['main_process_port']}"
    if cfg["rdzv_backend"] == "static" and int(cfg["max_restarts"]) == 0:
        cmd += [f"--node-rank={cfg['machine_rank']}", f"--master-addr={cfg['main_process_ip']}",
                f"--master-port={cfg['main_process_port']}", "--rdzv-backend=static"]
    else:
        # restarts: the c10d rendezvous re-forms the group (fresh store keys per attempt); a static store
        # reused across attempts leaves stale gloo/RCCL connection keys behind
        backend = "c10d" if cfg["rdzv_backend"] == "static" else cfg["rdzv_backend"]
        cmd += [f"--rdzv-backend={backend}", f"--rdzv-endpoint={endpoint}", "--rdzv-id=pva"]
        if nnodes <= 1:
            cmd += ["--local-addr=127.0.0.1"] if cfg["main_process_ip"] in ("127.0.0.1", "localhost") else []
    if a.module:
        cmd.append("--module")
        target = target[1:]
    return cmd + target, env


def main(argv: Optional[List[str]] = None) -> int:
    a, _ = parse(sys.argv[1:] if argv is None else argv)
    cfg = resolve(a)
    cmd, env = build_command(a, cfg)
    proc = subprocess.Popen(cmd, env=env)
    try:
        return proc.wait()
    except KeyboardInterrupt:
        proc.terminate()
        return proc.wait()


if __name__ == "__main__":
    sys.exit(main())
