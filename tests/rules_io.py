"""Golden rule-audit vectors (tests/golden/rules_*.json.gz, made by make_rules_golden.py)."""
import glob
import os
from collections import OrderedDict

import numpy as np

from golden_io import GOLDEN, dense, load

RULE_POOLS = sorted(os.path.basename(p)[:-8] for p in glob.glob(os.path.join(GOLDEN, "rules_*.json.gz")))


def ref_puzzle(p):
    """A processed puzzle in the reference's own format, rebuilt from a golden record."""
    obs = OrderedDict((k, dense(p["base"][k], np.int32)) for k in p["base_keys"])
    shapes = None
    if p["polyshapes"] is not None:
        shapes = {(int(k) if t == "int" else k): v for k, t, v in p["polyshapes"]}
    return {"x_size": p["x_size"], "y_size": p["y_size"], "obs_array": obs,
            "color_array": dense(p["color"], np.int32), "additional_info": dense(p["additional_info"], np.int64),
            "polyshapes": shapes, "target_location": tuple(p["target"]), "start_location": tuple(p["start"])}


def snapshots(g):
    """(episode, puzzle index, step number (-1 = reset), snapshot) over a golden pool."""
    for e, ep in enumerate(g["episodes"]):
        yield e, ep["puzzle_index"], -1, ep["reset"]
        for t, s in enumerate(ep["steps"]):
            yield e, ep["puzzle_index"], t, s
