"""One process per GPU from a single command.

The reference trains on every visible GPU from one ``python main.py``: ``load_ldm`` wraps the
UNet/VAE in ``DataParallel`` over ``torch.cuda.device_count()`` GPUs and returns that count
(``unsupervised_keypoints/optimize_token.py:42-50, 70, 79``).  Here the same command starts one
rank per GPU under ``torch.distributed.run`` (RCCL over xGMI) and exits with its status.

The parent must not have touched HIP (a process that initialised the GPU may not be replaced, and
its children would inherit nothing useful): it only counts devices, which on this image does not
initialise the runtime, and starts the launcher as a CHILD process (never ``os.exec*``).
"""
import os
import socket
import subprocess
import sys


def launcher_env():
    """(world, rank, local_rank) from the torch.distributed.run environment, or None outside it."""
    if "WORLD_SIZE" not in os.environ:
        return None
    return (int(os.environ["WORLD_SIZE"]), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")))


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(nproc, target, argv, env=None):
    """Run ``target`` (a script path, or ``-m module``) with ``argv`` as ``nproc`` ranks of
    ``python -m torch.distributed.run`` on this node (rendezvous on 127.0.0.1); returns the exit
    status of the launcher.  ``target`` is a list: ``[path]`` or ``["-m", "pkg.mod"]``."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}"] + list(target) + list(argv)
    full_env = dict(os.environ if env is None else env)
    full_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver (RCCL)
    return subprocess.run(cmd, env=full_env).returncode
