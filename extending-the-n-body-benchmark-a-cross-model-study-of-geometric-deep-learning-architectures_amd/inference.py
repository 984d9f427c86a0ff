"""Self-feed rollout API — drop-in for helper_scripts/infer_self_feed.py:20-254
(``run_inference``), the self_feed.py names the trainer imports (``SelfFeedError``,
``MACROS_DIR_NAME``, self_feed.py:25-40) and Trainer.run_self_feed's energy
post-processing (trainer.py:888-1010).

``run_inference`` keeps the reference's signature, seeding, dataset handling,
truncation, output arrays ([2, B, T, N, 3]: ground truth, prediction) and
``.npy`` file layout, but the rollout itself is ONE device-resident call
(``model.rollout``): graph, features, forward and state update stay in HBM for all
T-1 steps and the trajectory comes back to the host once, instead of a Python
loop with a device->host copy per step.  Models compute in fp32 on the device;
the returned predictions are cast to the dataset precision like the reference's.
Macro plotting (``plot_macros``) is outside the native scope and is ignored with
a warning.
"""
from __future__ import annotations

import json
import inspect
import os
import re
import warnings
from datetime import datetime

import numpy as np
import torch

from . import _lib
from .dataloaders import get_device
from .dataset import GravityDatasetOtf

__all__ = ["run_inference", "load_model_for_inference", "SelfFeedError", "MACROS_DIR_NAME", "STEPS_TO_RETURN_MULTIPLIER", "nbody_energies",
           "get_dataset_metadata_path", "load_dataset_from_metadata_file", "SelfFeedTrainer"]

MACROS_DIR_NAME = "visualize_macros"
STEPS_TO_RETURN_MULTIPLIER = 100
NATIVE_MODEL_TYPES = ("segnn", "ponita", "egnn_mc", "equiformer_v2")


class SelfFeedError(RuntimeError):
    """self_feed.py:29-40."""

    def __init__(self, steps_survived: int):
        super().__init__(f"Self-feed failed after {steps_survived} steps")
        self.steps_survived = steps_survived


def get_dataset_metadata_path(path):
    """utils/nbody_utils.py:1452-1488: <highest run dir named YYYY-MM-DD_HH-MM-SS>/nbody_small_dataset/metadata.json."""
    current = os.path.abspath(path)
    pattern = re.compile(r"\d{4}-\d{2}-\d{2}_\d{2}-\d{2}-\d{2}")
    run_root = None
    while True:
        if pattern.match(os.path.basename(current)):
            run_root = current
        parent = os.path.dirname(current)
        if parent == current:
            break
        current = parent
    if run_root is None:
        raise FileNotFoundError("Run directory root not found")
    return os.path.join(run_root, "nbody_small_dataset", "metadata.json")


_DATASET_ARGS = ("dataset_name", "target", "path", "batch_size", "sim_length", "sample_freq", "noise_var",
                 "num_nodes", "vel_norm", "interaction_strength", "dt", "softening", "double_precision",
                 "center_of_mass", "lmax_attr", "use_cached", "cache_data")


def load_dataset_from_metadata_file(metadata_file_path, n_bodies=None, device=None, metadata=None):
    """datasets/nbody/visualization_utils.py:1438-1452: keep only constructor
    arguments (so the saved ``n_balls`` is NOT applied — num_nodes falls back to 5
    unless ``n_bodies`` is given, as in the reference)."""
    if metadata is None:
        with open(metadata_file_path) as f:
            metadata = json.load(f)
    kw = {k: metadata[k] for k in _DATASET_ARGS if k in metadata}
    if n_bodies is not None:
        kw["num_nodes"] = n_bodies
    return GravityDatasetOtf(device=device, **kw)


def nbody_energies(loc, vel, G, softening, device=None):
    """Trainer._compute_nbody_energies (trainer.py:888-927) on the device:
    loc/vel [B, T, N, 3] -> dict of batch-mean potential / kinetic / total [T] (numpy)."""
    device = device or get_device()
    l = torch.as_tensor(np.asarray(loc), dtype=torch.float64).to(device).contiguous()
    v = torch.as_tensor(np.asarray(vel), dtype=torch.float64).to(device).contiguous()
    B, T, N, _ = l.shape
    kin = torch.empty(B, T, dtype=torch.float64, device=device)
    pot = torch.empty_like(kin)
    mk = torch.empty(T, dtype=torch.float64, device=device)
    mp = torch.empty_like(mk)
    _lib.check(_lib.lib().nbx_nbody_energies(_lib.dev_ptr(l), _lib.dev_ptr(v), B, T, N, float(G), float(softening),
                                             _lib.dev_ptr(kin), _lib.dev_ptr(pot), _lib.dev_ptr(mk), _lib.dev_ptr(mp),
                                             _lib.stream_ptr(device)), "nbx_nbody_energies")
    mk, mp = mk.cpu().numpy(), mp.cpu().numpy()
    return {"potential": mp, "kinetic": mk, "total": mp + mk}


def load_model_for_inference(model_path, model_type, device):
    """utils/nbody_utils.py:1316-1373 + load_checkpoint (:1376-1407): the family's default
    constructor, the checkpoint's ``model_state_dict`` (or a bare state_dict), then
    ``eval()`` on ``device``.  Checkpoints are read with ``torch.load(weights_only=True)``
    (tensors and plain containers only).  Like the reference: equiformer(_v2), segnn, ponita."""
    from .equiformer_v2 import EquiformerV2_nbody
    from .ponita import PONITA_NBODY
    from .segnn import SEGNN
    print(f"Initializing model of type '{model_type}' on device {device}")
    if model_type == "equiformer":
        model = EquiformerV2_nbody(device)
    elif model_type == "equiformer_v2":   # nbody_utils.py:1324-1361
        model = EquiformerV2_nbody(
            device=device, use_pbc=False, regress_forces=True, otf_graph=True, max_neighbors=5, max_radius=4096.0,
            max_num_elements=90, num_layers=3, attn_hidden_channels=32, sphere_channels=32, num_heads=2,
            attn_alpha_channels=8, attn_value_channels=4, ffn_hidden_channels=64, norm_type="rms_norm_sh",
            lmax_list=[2], mmax_list=[1], grid_resolution=None, num_sphere_samples=32, edge_channels=32,
            use_atom_edge_embedding=True, share_atom_edge_embedding=False, use_m_share_rad=False,
            distance_function="projection", num_distance_basis=64, attn_activation="scaled_silu",
            use_s2_act_attn=False, use_attn_renorm=True, ffn_activation="scaled_silu", use_gate_act=False,
            use_grid_mlp=False, use_sep_s2_act=True, alpha_drop=0.01, drop_path_rate=0.0, proj_drop=0.0,
            weight_init="normal")
    elif model_type == "segnn":
        model = SEGNN()
    elif model_type == "ponita":
        model = PONITA_NBODY()
    else:
        raise ValueError(f"Unsupported model_type: {model_type}")
    print(f"Loading checkpoint from {model_path} on device {device}")
    ckpt = torch.load(model_path, map_location="cpu", weights_only=True)
    if isinstance(ckpt, dict) and "model_state_dict" in ckpt:
        model.load_state_dict(ckpt["model_state_dict"])
    elif isinstance(ckpt, dict) and all(isinstance(v, torch.Tensor) for v in ckpt.values()):
        model.load_state_dict(ckpt)
    else:
        raise ValueError("Checkpoint does not contain a model state dict.")
    model.eval().to(device)
    return model


@torch.no_grad()
def run_inference(model_type, dataloader, model_path=None, model=None, save_dir=None, print_step=True, n_bodies=None,
                  plot_macros=False, num_neighbors=None, device=None, max_rollout_steps=None, dataset=None,
                  shard=None):
    """infer_self_feed.py:20-254.  Returns ``(trajectories_save_dir,
    combined_locations [2,B,T,N,3], combined_velocities [2,B,T,N,3])``.

    The dataset comes from ``dataset`` if given, else from the run's metadata file
    (``model_path``), else from the dataloader's dataset attributes.  ``model=None``
    loads ``model_path`` like the reference (load_model_for_inference).

    ``shard`` (default: on when torch.distributed has more than one rank): one process
    per GPU, each rank integrates the ground truth of its contiguous block of the B
    systems and rolls it out; a SEGNN in train mode keeps the reference's full-batch
    BatchNorm statistics through SyncBN (12 all-reduces of 288 doubles per step); one
    all-gather at the end assembles the [2, B, T, N, 3] arrays on every rank and rank 0
    writes the files."""
    from . import parallel as P
    torch.manual_seed(42)
    if device is None:
        device = get_device()
    device = torch.device(device)
    if model_type not in NATIVE_MODEL_TYPES:
        raise ValueError(f"model_type {model_type!r} has no native rollout (native: {NATIVE_MODEL_TYPES})")
    if dataset is None:
        meta = None
        if model_path is not None:
            try:
                meta_path = get_dataset_metadata_path(model_path)
                if os.path.exists(meta_path):
                    with open(meta_path) as f:
                        meta = json.load(f)
            except FileNotFoundError:
                meta = None
        if meta is None:
            if dataloader is None:
                raise FileNotFoundError("no dataset metadata next to model_path and no dataloader given")
            meta = dataloader.dataset.get_serializable_attributes()
            meta.setdefault("num_nodes", meta.get("n_balls"))
            if n_bodies is None:
                n_bodies = meta["num_nodes"]
        dataset = load_dataset_from_metadata_file(None, n_bodies=n_bodies, device=device, metadata=meta)
    if model is None:
        if model_path is None:
            raise ValueError("run_inference needs a model or a model_path")
        model = load_model_for_inference(model_path, model_type, device)
    model = model.double() if dataset.double_precision else model.float()

    world = P.world()
    shard = (world > 1) if shard is None else (bool(shard) and world > 1)
    batch_size = dataset.batch_size
    if shard:
        start, count = P.shard_range(batch_size, P.rank(), world)
        batch_data, _ = dataset.get_ground_truth_trajectories(batch_size=count, shard=False)
    else:
        count = batch_size
        batch_data, _ = dataset.get_ground_truth_trajectories(batch_size=batch_size)
    loc_actual, vel_actual, force_actual, mass_actual = [torch.from_numpy(np.array(d)) for d in zip(*batch_data)]
    output_dims = loc_actual.shape[-1]
    n_nodes = loc_actual.shape[-2]
    num_neighbors = num_neighbors if num_neighbors is not None else n_nodes - 1
    knn = {}
    if model_type in ("segnn", "ponita"):   # the branches that build_graph_with_knn (lines 121-123, 137-139)
        if num_neighbors >= n_nodes:
            raise ValueError("Graph cannot have more neighbors than there are nodes in simulation - 1")
        if num_neighbors != n_nodes - 1:
            if "num_neighbors" not in inspect.signature(model.rollout).parameters:
                raise NotImplementedError(f"native {model_type} rollout: kNN graphs (num_neighbors < N-1) "
                                          "are not supported")
            knn = {"num_neighbors": int(num_neighbors)}
    elif model_type == "egnn_mc":
        # lines 161-170: the graph comes from dataloader.preprocess_batch, i.e. the dataloader's own
        # args.num_neighbors (egnn_mc_n_body_dataloader.py:13-19: None / <= 0 / >= N: fully connected)
        k = getattr(getattr(dataloader, "args", None), "num_neighbors", None)
        if k is not None and 0 < int(k) < n_nodes - 1:
            knn = {"num_neighbors": int(k)}
    num_steps = loc_actual.shape[1]
    if max_rollout_steps is not None:
        try:
            max_rollout_steps = int(max_rollout_steps)
            if max_rollout_steps > 0:
                num_steps = min(num_steps, max_rollout_steps)
                loc_actual = loc_actual[:, :num_steps]
                vel_actual = vel_actual[:, :num_steps]
        except Exception as e:  # reference: print and keep the full length
            print(e)
    print(f"Number of steps to generate: {num_steps}")

    dtype = torch.float64 if dataset.double_precision else torch.float32
    loc0 = loc_actual[:, 0].to(device=device, dtype=dtype)
    vel0 = vel_actual[:, 0].to(device=device, dtype=dtype)
    mass0 = mass_actual.reshape(count, n_nodes, 1).to(device=device, dtype=dtype)
    if print_step:
        print(f"Predicting {num_steps - 1} steps for {batch_size} simulations (device-resident rollout"
              + (f", {count} on rank {P.rank()} of {world})" if shard else ")"))
    # infer_self_feed.py:185-186: only "pos_dt+vel" adds the prediction to the previous position
    kw = {"absolute": True} if dataset.target != "pos_dt+vel" else {}
    kw.update(knn)
    sync = shard and hasattr(model, "enable_sync_batchnorm") and model.training
    if sync:
        model.enable_sync_batchnorm(global_batch=batch_size)   # no per-call batch-size collective
    # PONITA's one-time calibration (conv.py:134-140) from the moments of the whole sharded batch
    calib = shard and hasattr(model, "calibration_group") and model.calibration_group is None
    if calib:
        import torch.distributed as dist
        model.calibration_group = dist.group.WORLD
    try:
        tp, tv = model.rollout(loc0, vel0, mass0, num_steps, **kw)
    finally:
        if sync:
            model.disable_sync_batchnorm()
        if calib:
            model.calibration_group = None
    print("Finished prediction for all simulations")
    steps_in_actual = loc_actual.shape[1]
    loc_actual = loc_actual.reshape(count, steps_in_actual, n_nodes, output_dims)
    vel_actual = vel_actual.reshape(count, steps_in_actual, n_nodes, output_dims)
    if shard:   # the one collective of the sharded rollout: [count, T, N, 3] x 4 -> [B, T, N, 3] x 4
        gt = [t.to(device=device, dtype=loc_actual.dtype).contiguous() for t in (loc_actual, vel_actual)]
        loc_actual, vel_actual = (P.all_gather_shards(t, batch_size) for t in gt)
        tp, tv = (P.all_gather_shards(t.contiguous(), batch_size) for t in (tp, tv))
    loc_pred = tp.to(dtype).cpu().numpy()
    vel_pred = tv.to(dtype).cpu().numpy()
    loc_actual = loc_actual.cpu().numpy() if torch.is_tensor(loc_actual) else loc_actual
    vel_actual = vel_actual.cpu().numpy() if torch.is_tensor(vel_actual) else vel_actual
    combined_locations = np.stack([loc_actual, loc_pred], axis=0)
    combined_velocities = np.stack([vel_actual, vel_pred], axis=0)

    if not save_dir:
        base = os.path.dirname(model_path) if model_path else "."
        save_dir = f"{base}/generated_trajectories/{datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}"
    out_dir = os.path.join(save_dir, "trajectories_data")
    if P.rank() == 0 or not shard:
        os.makedirs(save_dir, exist_ok=True)
        if plot_macros:
            warnings.warn("plot_macros is outside the native rollout scope; skipped")
        os.makedirs(out_dir, exist_ok=True)
        for i in range(batch_size):
            np.save(os.path.join(out_dir, f"loc_actual_sim_{i}.npy"), loc_actual[i])
            np.save(os.path.join(out_dir, f"loc_pred_sim_{i}.npy"), loc_pred[i])
            np.save(os.path.join(out_dir, f"vel_actual_sim_{i}.npy"), vel_actual[i])
            np.save(os.path.join(out_dir, f"vel_pred_sim_{i}.npy"), vel_pred[i])
        print(f"Saved actual and predicted trajectories for all simulations to {out_dir}")
    if shard:
        P.barrier()
    return out_dir, combined_locations, combined_velocities


class SelfFeedTrainer:
    """The self-feed half of trainer.Trainer (trainer.py:929-1010): ``run_self_feed``
    rolls the model out with ``run_inference`` and computes the energy series on the
    device.  Training itself is outside the native path."""

    def __init__(self, model, train_dataloader, validation_dataloader=None, args=None, save_dir_path="."):
        self.model, self.dataloader, self.args = model, train_dataloader, args
        self.save_dir_path = save_dir_path
        self.step_count = 1
        self.device = train_dataloader.device if train_dataloader is not None else get_device()
        self.last_energies = None

    def _compute_nbody_energies(self, loc, vel, G, softening):
        return nbody_energies(loc, vel, G, softening, self.device)

    def run_self_feed(self):
        print(f"Running self feed (epoch {self.step_count - 1})")
        max_steps = getattr(self.args, "self_feed_limit_steps", None)
        _, locs, vels = run_inference(model_type=self.args.model_type, dataloader=self.dataloader,
                                      model_path=None, model=self.model,
                                      save_dir=f"{self.save_dir_path}/checkpoints/{self.step_count}",
                                      print_step=True, device=self.device, max_rollout_steps=max_steps)
        steps = locs.shape[2] - 1
        sim = self.dataloader.dataset.simulation
        G, soft = float(sim.interaction_strength), float(sim.softening)
        self.last_energies = {"simulation": self._compute_nbody_energies(locs[0], vels[0], G, soft),
                              "self_feed": self._compute_nbody_energies(locs[1], vels[1], G, soft)}
        self.self_feed_postprocess_common(energies=self.last_energies, steps_survived=steps,
                                          save_dir=f"{self.save_dir_path}/checkpoints/{self.step_count}",
                                          metrics_filename="nbody_macro_metrics.json")
        return steps

    def self_feed_postprocess_common(self, *, energies, steps_survived, save_dir,
                                     metrics_filename="nbody_macro_metrics.json"):
        """trainer.py:668-779 for the N-body energies: steps within the energy-ratio
        thresholds, KS p-values of the energy series (device statistics, ks.py) and their
        Fisher combination, persisted as ``metrics_filename`` in the reference's JSON layout.
        W&B logging and plotting are outside the native scope; the results are kept in
        ``self.last_macros``."""
        from .ks import energy_steps_within, macro_pvalues
        os.makedirs(save_dir, exist_ok=True)
        steps_metric = energy_steps_within(energies["simulation"]["total"], energies["self_feed"]["total"])
        print("Self feed energy within " + "| ".join(f"{t * 100:.0f}%: {n} steps" for t, n in steps_metric.items()))
        pvals, p_combined = macro_pvalues(energies)
        f = lambda v: float(v) if v == v else float("nan")
        to_json = {
            "energies": {f"{src}_{k}": np.asarray(energies[side][k]).tolist()
                         for src, side in (("simulation", "simulation"), ("self_feed", "self_feed"))
                         for k in ("total", "potential", "kinetic")},
            "ks_pvalues": {**{k: f(v) for k, v in pvals.items()}, "combined": f(p_combined)},
        }
        with open(os.path.join(save_dir, metrics_filename), "w") as fh:
            json.dump(to_json, fh)
        self.last_macros = {"steps_within": steps_metric, "ks_pvalues": pvals, "ks_combined": p_combined,
                            "steps_survived": int(steps_survived)}
        return steps_metric
