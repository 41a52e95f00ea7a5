"""Measured GEMM solution choices for the frozen SD UNet / VAE (PyTorch TunableOp, read-only).

``gemm_gfx950.csv`` holds, for every hipBLASLt / rocBLAS GEMM shape of the token-opt step at
the BASELINE config, the solution TunableOp measured fastest on an MI355X (tools/tune_gemms.sh
regenerates it: one bench run with tuning on, ≈3 min).  Loading it swaps each listed GEMM's
heuristic kernel choice for the measured one — the same arithmetic (fp32 in, fp32 accumulate),
a different kernel and reduction order — and leaves unlisted shapes on the default path.  The
file's validator lines pin PyTorch / HIP / hipBLASLt / rocBLAS versions and the gfx950 arch; on
any mismatch it is not used.  ``SKP_TUNED_GEMMS=0`` disables it; ``SKP_TUNED_GEMMS_FILE``
names another results file (A/B of a re-tuning).

Scope: TunableOp's results table is **process-global** (one tuning context per process, keyed by
GEMM signature, not by device).  With one process per GPU — the only multi-GPU layout here —
rank k loads the file once for its own ``cuda:k``; the validators are checked against that
device (the file is read with it current), and ``use_tuned_gemms`` refuses to report the table as
in use on a device whose arch is not the file's.
"""
import os

import torch

TUNED_GEMMS = os.environ.get("SKP_TUNED_GEMMS_FILE") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                     "gemm_gfx950.csv")
TABLE_ARCH = "gfx950"
_state = {"loaded": None, "devices": set()}


def _arch(dev):
    return torch.cuda.get_device_properties(dev).gcnArchName.split(":")[0]


def use_tuned_gemms(device=None, path=None):
    """Enable TunableOp with tuning off and the measured results of ``path`` (read once per
    process, with ``device`` current); True if the table is in use for ``device``."""
    path = path or TUNED_GEMMS
    if not torch.cuda.is_available():
        return False
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if _state["loaded"] is None:
        ok = False
        if os.environ.get("SKP_TUNED_GEMMS", "1") != "0" and os.path.exists(path) and _arch(dev) == TABLE_ARCH:
            t = torch.cuda.tunable
            with torch.cuda.device(dev):
                t.set_filename(os.devnull)     # nothing is written back at exit
                t.tuning_enable(False)
                t.enable(True)
                ok = bool(t.read_file(path))
                if not ok:
                    t.enable(False)
        _state["loaded"] = ok
    ok = bool(_state["loaded"]) and _arch(dev) == TABLE_ARCH
    if ok:
        _state["devices"].add(dev.index)
    return ok


def tuned_devices():
    """Device indices of this process for which the tuned table was reported in use."""
    return sorted(_state["devices"])
