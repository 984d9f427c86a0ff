"""``python -m nbody_amd.self_feed [--config cfg.yaml] [--model_type ...] [--limit_steps K]``

The self_feed.py entry point for N-body (self_feed.py:413-435): build the model
and dataloader from the plugin registry, run the device-resident
``run_inference`` rollout capped at ``limit_steps`` (default 2000, as the
reference) and report the energy drift of the prediction against the ground
truth.  Prints one JSON summary line.
"""
from __future__ import annotations

import argparse
import json
import sys

import numpy as np

from .inference import MACROS_DIR_NAME, SelfFeedError, SelfFeedTrainer  # noqa: F401  (re-exported names)
from .registry import create_model, load_class_from_args, parse_args


def main(argv=None):
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--limit_steps", type=int, default=2000)
    pre.add_argument("--save_dir", default="self_feed_out")
    known, rest = pre.parse_known_args(argv)
    args, _ = parse_args(rest)
    args.self_feed_limit_steps = known.limit_steps
    model = create_model(args)
    dataloader = load_class_from_args(args, "dataloader")(args, partition="train")
    model = model.to(dataloader.device)
    trainer = SelfFeedTrainer(model, dataloader, args=args, save_dir_path=known.save_dir)
    steps = trainer.run_self_feed()
    e = trainer.last_energies
    drift = lambda s: float(np.abs(s["total"] - s["total"][0]).max())
    summary = {"model_type": args.model_type, "steps_survived": steps,
               "energy_drift_simulation": drift(e["simulation"]), "energy_drift_self_feed": drift(e["self_feed"])}
    print(json.dumps(summary), flush=True)
    return summary


if __name__ == "__main__":
    main(sys.argv[1:])
