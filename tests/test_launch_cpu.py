"""Launcher (accelerate-launch equivalent) and elastic fault recovery on CPU/gloo."""
import os
import socket
import subprocess

import pytest
import sys

from pytorchvideo_accelerate_amd import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_config_file_and_cli_precedence(tmp_path):
    cfg = tmp_path / "cfg.yaml"
    cfg.write_text("compute_environment: LOCAL_MACHINE\ndistributed_type: MULTI_GPU\nnum_processes: 8\n"
                   "mixed_precision: fp16\nmain_process_port: 29600\ngpu_ids: all\n")
    a, _ = launch.parse(["--config_file", str(cfg), "--mixed_precision", "bf16", "run.py", "--is_slowfast"])
    c = launch.resolve(a)
    assert c["num_processes"] == 8 and c["mixed_precision"] == "bf16" and c["main_process_port"] == 29600
    cmd, env = launch.build_command(a, c)
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd
    assert cmd[-2:] == ["run.py", "--is_slowfast"] and env["ACCELERATE_MIXED_PRECISION"] == "bf16"
    # one process: plain child process, script args untouched
    a, _ = launch.parse(["--num_processes", "1", "--cpu", "run.py", "--lr", "0.5"])
    cmd, env = launch.build_command(a, launch.resolve(a))
    assert cmd == [sys.executable, "run.py", "--lr", "0.5"] and env["ACCELERATE_USE_CPU"] == "true"


def test_default_process_count_is_visible_gpus(tmp_path, monkeypatch):
    """accelerate without a config file (the reference's bare ``accelerate launch run.py``): one rank per GPU,
    also for ``--multi_gpu`` without ``--num_processes`` ([acc] commands/launch.py:1302-1340)."""
    monkeypatch.setenv("ACCELERATE_CONFIG_FILE", str(tmp_path / "absent.yaml"))
    monkeypatch.setattr(launch, "_device_count", lambda: 8)
    for argv in (["--multi_gpu", "run.py", "--is_slowfast"], ["run.py", "--is_slowfast"]):
        a, _ = launch.parse(argv)
        c = launch.resolve(a)
        cmd, _ = launch.build_command(a, c)
        assert c["num_processes"] == 8 and c["distributed_type"] == "MULTI_GPU"
        assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd, cmd
    # explicit count, CPU runs and a config file keep their own count
    a, _ = launch.parse(["--num_processes", "1", "run.py"])
    assert launch.build_command(a, launch.resolve(a))[0] == [sys.executable, "run.py"]
    a, _ = launch.parse(["--cpu", "run.py"])
    assert launch.resolve(a)["num_processes"] == 1
    cfg = tmp_path / "cfg.yaml"
    cfg.write_text("distributed_type: NO\nmixed_precision: bf16\n")
    a, _ = launch.parse(["--config_file", str(cfg), "run.py"])
    assert launch.resolve(a)["num_processes"] == 1
    # the env-mask count never starts a child process
    monkeypatch.undo()
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    assert launch._device_count() == 4


def test_fault_injection_elastic_restart_auto_resume(tmp_path):
    """Both ranks fail after global step 3; torchrun restarts the group; --auto_resume continues from step_2."""
    out = tmp_path / "out"
    cmd = [sys.executable, "-m", "pytorchvideo_accelerate_amd.launch", "--cpu", "--num_processes", "2",
           "--max_restarts", "1", "--monitor_interval", "1", "--main_process_port", str(_port()), "--auto_resume",
           os.path.join(REPO, "run.py"), "--synthetic", "--synthetic_videos", "8", "--synthetic_classes", "3",
           "--num_frames", "8", "--crop_size", "64", "--batch_size", "2", "--num_workers", "0", "--num_epochs", "2",
           "--limit_val_batches", "0", "--checkpointing_steps", "2", "--output_dir", str(out),
           "--gradient_accumulation_steps", "1", "--quiet", "--logging_dir", str(tmp_path / "logs")]
    env = dict(os.environ, PVA_FAULT="step=3", OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="", PYTHONPATH=REPO)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=str(tmp_path), env=env)
    log = r.stdout[-4000:] + r.stderr[-4000:]
    assert r.returncode == 0, log
    assert "injected fault at global step 3" in log and "Resumed from checkpoint" in log
    assert (out / ".fault_injected_0").exists() and (out / ".fault_injected_1").exists()
    assert (out / "step_4" / "model.safetensors").exists()  # 2 epochs x 2 global steps; final save


@pytest.mark.parametrize("nproc", [1, 2])
def test_crash_inside_checkpoint_save_restarts_from_previous(tmp_path, nproc):
    """The elastic agent restarts a run whose step-4 save died half-way; --auto_resume continues from the complete
    step_2 checkpoint (not the partial step_4.tmp) and the run finishes.  With 2 ranks only the main process
    crashes (it alone writes the shared files) while rank 1 waits in the save's barrier: the agent tears the whole
    group down on the main process's exit (no collective timeout) and restarts it."""
    out = tmp_path / "out"
    cmd = [sys.executable, "-m", "pytorchvideo_accelerate_amd.launch", "--cpu", "--num_processes", str(nproc),
           "--max_restarts", "1", "--monitor_interval", "1", "--main_process_port", str(_port()), "--auto_resume",
           os.path.join(REPO, "run.py"), "--synthetic", "--synthetic_videos", "8", "--synthetic_classes", "3",
           "--num_frames", "8", "--crop_size", "64", "--batch_size", "2", "--num_workers", "0", "--num_epochs", "2",
           "--limit_val_batches", "0", "--checkpointing_steps", "2", "--output_dir", str(out),
           "--gradient_accumulation_steps", "1", "--quiet", "--logging_dir", str(tmp_path / "logs")]
    env = dict(os.environ, PVA_FAULT="save=4", OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="", PYTHONPATH=REPO)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=str(tmp_path), env=env)
    log = r.stdout[-4000:] + r.stderr[-4000:]
    assert r.returncode == 0, log
    assert "injected fault while saving" in log and "Resumed from checkpoint" in log and "step_2" in log, log
    assert (out / ".save_fault_injected_0").exists()
    assert (out / f"step_{8 // nproc}" / ".pva_complete").exists() and not (out / "step_4.tmp").exists()
