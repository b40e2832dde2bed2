"""Measured parity errors of the GPU step tests, appended as JSON lines to $SIREN_ERRLOG when
it is set (tools / DESIGN.md tables); the tolerances the tests assert are set from these."""
import json
import os

import numpy as np

STEP_TOL = 2e-3   # whole-step gradients vs the fp16-storage oracle (relative L2)


def rel(a, b) -> float:
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


def log(test: str, **vals) -> None:
    path = os.environ.get("SIREN_ERRLOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"test": test, **vals}) + "\n")


def check_grads(test: str, got: dict, ref: dict, tol: float = STEP_TOL) -> float:
    """max over parameters of rel(got, ref); logs every value, then asserts each < tol."""
    errs = {k: rel(got[k].reshape(r.shape), r) for k, r in ref.items()}
    worst = max(errs.values())
    log(test, worst=worst, errs=errs)
    for k, e in errs.items():
        assert e < tol, (test, k, e)
    return worst
