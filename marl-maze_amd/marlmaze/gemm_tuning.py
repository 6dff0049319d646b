"""Pre-tuned GEMM selection for the actor/critic GEMMs (PyTorch TunableOp).

The MLP GEMMs of the PPO update are plain fp32 library GEMMs (hipBLASLt /
rocBLAS).  For the skinny shapes of this workload (M = 419,430 rows,
N, K in {6, 64, 130, 264, 460}) the libraries' default heuristics pick tiles
that reach ~50% of the fp32 MFMA peak; TunableOp times every candidate
solution once and records the fastest per shape.  ``tuned/gemm_gfx950.csv``
holds those records for the bench workload (65,536 mazes x 16 steps per GPU;
the per-rank shapes are the same at every world size), produced by
``tools/tune_gemms.sh`` on an MI355X.  Loading it only changes which library
kernel runs (same fp32 arithmetic, a different summation order); shapes that
are not in the file use the default heuristic.  Tuning itself stays off.
"""
import os
import tempfile

import torch

TUNED_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "gemm_gfx950.csv")


def enable_tuned_gemms(path=TUNED_FILE):
    """Turn TunableOp on in lookup-only mode with the shipped results.
    Returns True when the file was read."""
    if not torch.cuda.is_available() or not os.path.exists(path):
        return False
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(False)
    # TunableOp's own output file (never written while tuning is off) must not
    # be the shipped file
    t.set_filename(os.path.join(tempfile.gettempdir(), f"marlmaze_tunableop_{os.getpid()}.csv"))
    return bool(t.read_file(path))
