"""Measured GEMM solution choices for the frozen SD UNet / VAE (PyTorch TunableOp, read-only).

``gemm_gfx950.csv`` holds, for every hipBLASLt / rocBLAS GEMM shape of the token-opt step at
the BASELINE config, the solution TunableOp measured fastest on an MI355X (tools/tune_gemms.sh
regenerates it: one bench run with tuning on, ≈3 min).  Loading it swaps each listed GEMM's
heuristic kernel choice for the measured one — the same arithmetic (fp32 in, fp32 accumulate),
a different kernel and reduction order — and leaves unlisted shapes on the default path.  The
file's validator lines pin PyTorch / HIP / hipBLASLt / rocBLAS versions and the gfx950 arch; on
any mismatch it is not used.  ``SKP_TUNED_GEMMS=0`` disables it; ``SKP_TUNED_GEMMS_FILE``
names another results file (A/B of a re-tuning).
"""
import os

import torch

TUNED_GEMMS = os.environ.get("SKP_TUNED_GEMMS_FILE") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                     "gemm_gfx950.csv")
_state = {"loaded": None}


def use_tuned_gemms(path=TUNED_GEMMS):
    """Enable TunableOp with tuning off and the measured results of ``path``; True if in use."""
    if _state["loaded"] is not None:
        return _state["loaded"]
    ok = False
    if os.environ.get("SKP_TUNED_GEMMS", "1") != "0" and os.path.exists(path) and torch.cuda.is_available():
        t = torch.cuda.tunable
        t.set_filename(os.devnull)     # nothing is written back at exit
        t.tuning_enable(False)
        t.enable(True)
        ok = bool(t.read_file(path))
        if not ok:
            t.enable(False)
    _state["loaded"] = ok
    return ok
