"""GravityDatasetOtf — drop-in for datasets/nbody/dataset_gravity_otf.py:20-295
with the ground truth integrated on the device.

Same constructor, cache folder name (sha256 of the JSON of the constructor
arguments, lines 52-56,176-183), cache file format (``saved_simulations/<hash>/<k>.pkl``
holding a list of ``batch_size`` tuples ``(pos [T,N,3], vel, force, mass [N,1])``,
lines 118-135) and ``__getitem__`` targets (189-252), so caches written by either
side are interchangeable.  Differences, by design:

* ``get_ground_truth_trajectories`` integrates all ``batch_size`` systems in one
  HIP launch (csrc/gravity.hip) instead of a ProcessPool; trajectories come back in
  submission order rather than completion order.  Seeds are OS entropy as in the
  reference (``random_seed=None``) unless ``seeds`` is given.
* cached pickles are read with a restricted unpickler that accepts only numpy
  arrays, dtypes, lists and tuples — a cache file cannot execute code.
* plotting helpers (lines 297-716) are out of scope.
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import pathlib
import pickle
import random

import numpy as np
import torch

from .gravity import GravitySim

__all__ = ["GravityDatasetOtf", "load_cached_simulations", "save_cached_simulations"]


class _ArrayUnpickler(pickle.Unpickler):
    """Only what a list of numpy-array tuples needs."""

    _ALLOWED = {
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
        ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("builtins", "tuple"), ("builtins", "list"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a simulation cache")


def _log(msg):
    print(f"[GravityDatasetOtf] {msg}")


def load_cached_simulations(path):
    with open(path, "rb") as f:
        return _ArrayUnpickler(io.BytesIO(f.read())).load()


def save_cached_simulations(path, data):
    with open(path, "wb") as f:
        pickle.dump(data, f)


class GravityDatasetOtf:
    GROUND_TRUTH_FILE_PREFIXES = ["loc", "vel", "forces", "masses"]
    DEFAULT_DATA_PATH = os.path.join(pathlib.Path(__file__).parent.absolute(), "dataset", "gravity")

    def __init__(self, dataset_name="nbody_small", target="pos_dt+vel", path=DEFAULT_DATA_PATH, batch_size=8,
                 sim_length=10000, sample_freq=10, noise_var=0, num_nodes=5, vel_norm=1e-16,
                 interaction_strength=2, dt=0.01, softening=0.2, double_precision=False, center_of_mass=False,
                 lmax_attr=1, use_cached=False, cache_data=True, device=None, data_path="saved_simulations",
                 shard_generation=False):
        # the hash covers exactly the reference's constructor arguments (device / data_path /
        # shard_generation are ours)
        self.shard_generation = shard_generation
        self.locals = {"dataset_name": dataset_name, "target": target, "batch_size": batch_size,
                       "sim_length": sim_length, "sample_freq": sample_freq, "noise_var": noise_var,
                       "num_nodes": num_nodes, "vel_norm": vel_norm, "interaction_strength": interaction_strength,
                       "dt": dt, "softening": softening, "double_precision": double_precision,
                       "center_of_mass": center_of_mass, "lmax_attr": lmax_attr}
        self.cached_folder_name = self._get_cached_folder_name()
        self.data_path = data_path
        self.noise_var, self.num_nodes, self.vel_norm = noise_var, num_nodes, vel_norm
        self.interaction_strength, self.dt, self.softening = interaction_strength, dt, softening
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.simulation = self.init_simulation_instance()
        self.dataset_name, self.path, self.base_data_dir = dataset_name, path, path
        self.double_precision, self.center_of_mass, self.lmax_attr = double_precision, center_of_mass, lmax_attr
        self.use_cached, self.cache_data = use_cached, cache_data
        self.target = target
        self.sample_freq = sample_freq
        self.sim_length = sim_length - (sim_length % sample_freq)
        self.num_steps = sim_length // sample_freq
        self.batch_size = batch_size
        self.data_queue, self.unused_indices_queue = [], []
        self.cache_index = 0
        if use_cached:
            self._load_saved_simulations(self.cache_index)
        else:
            self._load_more_batches()

    # ------------------------------------------------------------ generation
    def init_simulation_instance(self):
        return GravitySim(noise_var=self.noise_var, n_balls=self.num_nodes, vel_norm=self.vel_norm,
                          interaction_strength=self.interaction_strength, dt=self.dt, softening=self.softening,
                          device=self.device)

    def get_ground_truth_trajectories(self, batch_size=None, seeds=None, shard=None):
        """lines 91-107: ``batch_size`` trajectories ``(pos, vel, force, mass)`` of
        ``sim_length / sample_freq`` frames, integrated in one device launch.  ``shard``
        (default: the constructor's ``shard_generation``): under torch.distributed each rank
        integrates its block of the trajectories and one all-gather assembles the batch on
        every rank (the reference's ProcessPool, lines 96-104, spread over GPUs)."""
        if batch_size is None:
            batch_size = self.batch_size
        shard = self.shard_generation if shard is None else shard
        batch_data = self.simulation.sample_trajectory_batch(batch_size, self.sim_length, self.sample_freq,
                                                             seeds=seeds, shard=shard)
        return batch_data, self.get_serializable_attributes()

    def _load_more_batches(self):
        """Integrate a fresh batch, queue it (all its frame pairs unused) and optionally cache it."""
        batch, _ = self.get_ground_truth_trajectories()
        self._enqueue(batch)
        if self.cache_data:
            self._save_simulations(batch)

    # ------------------------------------------------------------ cache
    def _cache_folder(self):
        return f"{self.data_path}/{self.cached_folder_name}"

    @staticmethod
    def _pickles(folder):
        return [fn for fn in os.listdir(folder) if fn.endswith(".pkl")]

    def _save_simulations(self, data):
        """Next free integer file name in the cache folder (<k>.pkl, k = 1 + the largest present)."""
        folder = self._cache_folder()
        os.makedirs(folder, exist_ok=True)
        taken = [int(fn[:-4]) for fn in self._pickles(folder)]
        path = f"{folder}/{max(taken) + 1 if taken else 0}.pkl"
        save_cached_simulations(path, data)
        _log(f"cached {len(data)} trajectories -> {path}")

    def _load_saved_simulations(self, index):
        """Queue cache file number ``index`` (sorted file names); when the folder is missing or the
        files are used up, switch to generation for good (cache_index = -1)."""
        folder = self._cache_folder()
        files = sorted(self._pickles(folder)) if os.path.exists(folder) else None
        if files is None or index >= len(files):
            _log(f"simulation cache {self.cached_folder_name}: "
                 + ("folder missing" if files is None else f"all {len(files)} files used") + "; generating")
            self.cache_index = -1
            self._load_more_batches()
            return
        _log(f"simulation cache {self.cached_folder_name}: reading file {index} ({files[index]})")
        self._enqueue(load_cached_simulations(f"{folder}/{files[index]}"))
        self.cache_index += 1

    def _enqueue(self, batch):
        frames = batch[0][0].shape[0]
        self.data_queue.append(batch)
        self.unused_indices_queue.append(list(range(frames - 1)))   # frame_0 candidates (frame_T = frame_0 + 1)

    # kept for callers of the reference's name
    _push_simulations_into_data_queue = _enqueue

    def _get_cached_folder_name(self):
        return hashlib.sha256(json.dumps(self.locals, sort_keys=True).encode()).hexdigest()

    # ------------------------------------------------------------ samples
    # target -> y from the batch arrays (loc / vel / force [B, T, N, 3]) and the frame pair; the first
    # two index the batch's FIRST axis with the frame number, exactly as the reference does
    _TARGETS = {
        "pos": lambda loc, vel, force, f0, fT: loc[fT],
        "force": lambda loc, vel, force, f0, fT: force[fT],
        "pos_dt+vel_dt": lambda loc, vel, force, f0, fT: np.concatenate((loc[fT] - loc[f0], vel[fT] - vel[f0]), axis=1),
        "pos_dt+vel": lambda loc, vel, force, f0, fT: np.concatenate((loc[:, fT] - loc[:, f0], vel[:, fT]), axis=2),
        "pos+vel": lambda loc, vel, force, f0, fT: np.concatenate((loc[:, fT], vel[:, fT]), axis=2),
        "pos_com+vel": lambda loc, vel, force, f0, fT: np.concatenate(
            (loc[fT] - np.mean(loc[f0], axis=0)[None, :], vel[fT]), axis=1),
    }

    def _advance_queue(self):
        """The head batch has no unused frame pair left: drop it; if the queue is then empty, refill
        it from the cache (while it lasts) or by generating."""
        _log("head simulation batch exhausted; moving to the next one")
        del self.data_queue[0], self.unused_indices_queue[0]
        if not self.unused_indices_queue:
            _log("simulation queue empty; refilling")
            if self.cache_index == -1:
                self._load_more_batches()
            else:
                self._load_saved_simulations(self.cache_index)

    def __getitem__(self, _):
        """One random unused frame pair (frame_0, frame_0 + 1) of the head batch (random.choice, then
        removed): (loc, vel, force at frame_0 [B, N, 3], mass, target)."""
        if not self.unused_indices_queue[0]:
            self._advance_queue()
        loc, vel, force, mass = (np.array(x) for x in zip(*self.data_queue[0]))
        f0 = random.choice(self.unused_indices_queue[0])
        self.unused_indices_queue[0].remove(f0)
        make = self._TARGETS.get(self.target)
        if make is None:
            raise Exception(f"Wrong target {self.target}")
        y = make(loc, vel, force, f0, f0 + 1)
        return (torch.tensor(loc[:, f0]), torch.tensor(vel[:, f0]), torch.tensor(force[:, f0]),
                torch.tensor(mass), torch.tensor(y))

    def get_serializable_attributes(self):
        return {"dataset_name": self.dataset_name, "target": self.target, "path": self.path,
                "batch_size": self.batch_size, "sim_length": self.sim_length, "sample_freq": self.sample_freq,
                "noise_var": self.noise_var, "n_balls": self.num_nodes, "vel_norm": self.vel_norm,
                "interaction_strength": self.interaction_strength, "dt": self.dt, "softening": self.softening,
                "double_precision": self.double_precision, "center_of_mass": self.center_of_mass}

    def get_one_sim_data(self, simulation_index):
        loc, vel, force, mass = (np.array(x) for x in zip(*self.data_queue[0]))
        return loc[simulation_index], vel[simulation_index], force[simulation_index], mass[simulation_index]
