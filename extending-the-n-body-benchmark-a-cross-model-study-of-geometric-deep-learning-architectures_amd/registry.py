"""The ``--model_type`` / ``--dataloader_type`` plugin registry with the native
models behind it — mirrors utils/config_models.py, utils/config.py:1-230 and
utils/utils_train.py:19-137 for the in-scope families (SEGNN, PONITA, EGNN-MC,
EquiformerV2 and their N-body dataloaders).

* ``MODEL_CONFIG_NAMES`` / ``DATALOADER_CONFIG_NAMES`` / ``TRAINER_CONFIG_NAMES``:
  name -> pydantic config; ``class_path`` must import (config_models.py:8-23).
* ``parse_args(argv)``: YAML config (``--config``, default ``config.yaml``) plus
  ``--section.key value`` overrides, flattened and stripped to the leaf names the
  reference's models read (later sections win on name clashes, as in the
  reference: the trainer's ``learning_rate`` shadows the model's).
* ``load_class_from_args(args, section)`` and ``create_model(args)`` as in
  utils_train.py.  Families outside the native path raise ``ValueError``.
"""
from __future__ import annotations

import argparse
import importlib
import os
from enum import Enum
from types import SimpleNamespace
from typing import Literal, Optional, Union

import yaml
from pydantic import BaseModel, Field, field_validator

__all__ = ["MODEL_CONFIG_NAMES", "DATALOADER_CONFIG_NAMES", "TRAINER_CONFIG_NAMES", "MainConfig", "PrecisionMode",
           "parse_args", "load_config", "load_class_from_args", "create_model", "DEFAULT_CONFIG_PATH"]

DEFAULT_CONFIG_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config.yaml")


def import_class(class_path: str):
    module_name, class_name = class_path.rsplit(".", 1)
    return getattr(importlib.import_module(module_name), class_name)


class BaseConfig(BaseModel):
    class_path: str = Field(..., description="Full path to the class, e.g. nbody_amd.segnn.SEGNN")
    model_config = {"protected_namespaces": (), "extra": "forbid"}

    @field_validator("class_path", mode="before")
    @classmethod
    def _importable(cls, v):
        import_class(v)          # raise early if the plugin does not import
        return v


class PonitaModelConfig(BaseConfig):
    name: Literal["ponita"] = "ponita"
    num_layers: int = 4
    hidden_features: int = 64
    learning_rate: float = 0.01


class SegnnModelConfig(BaseConfig):
    name: Literal["segnn"] = "segnn"
    lmax_attr: int = 1
    lmax_h: int = 1
    num_layers: int = 4
    hidden_features: int = 64
    model_type: str = "segnn"
    normalization_type: Optional[str] = None


class EgnnMcModelConfig(BaseConfig):
    name: Literal["egnn_mc"] = "egnn_mc"
    class_path: str = "nbody_amd.egnn_mc.EGNNMultiChannel"
    num_layers: int = 6
    hidden_node_dim: int = 192
    hidden_edge_dim: int = 192
    hidden_coord_dim: int = 128
    node_input_dim: int = 2
    edge_attr_dim: int = 4
    activation: str = "silu"
    coords_weight: float = 1.0
    recurrent: bool = True
    norm_diff: bool = False
    tanh: bool = False


class EquiformerV2ModelConfig(BaseConfig):
    """utils/config_models.py:56-81."""
    name: Literal["equiformer_v2"] = "equiformer_v2"
    class_path: str = "nbody_amd.equiformer_v2.EquiformerV2_nbody"
    use_pbc: bool = False
    max_neighbors: int = 5
    max_radius: float = 4096.0
    num_layers: int = 3
    attn_hidden_channels: int = 32
    sphere_channels: int = 32
    num_heads: int = 2
    attn_alpha_channels: int = 8
    attn_value_channels: int = 4
    ffn_hidden_channels: int = 64
    lmax_list: list = Field(default_factory=lambda: [2])
    mmax_list: list = Field(default_factory=lambda: [1])
    grid_resolution: Optional[int] = None
    edge_channels: int = 32
    use_atom_edge_embedding: bool = True
    share_atom_edge_embedding: bool = False
    distance_function: str = "projection"
    num_distance_basis: int = 64
    attn_activation: str = "scaled_silu"
    use_s2_act_attn: bool = False
    ffn_activation: str = "scaled_silu"


class GravityDatasetOtfConfig(BaseModel):
    dataset_name: str
    num_atoms: int = 5
    target: str = "pos_dt+vel"
    sample_freq: int = 10
    center_of_mass: bool = False
    interaction_strength: float = 2
    softening: float = 0.2


class PonitaNBodyDataLoaderConfig(BaseConfig):
    name: Literal["ponita_nbody"] = "ponita_nbody"
    num_neighbors: int
    batch_size: int = 128
    double_precision: bool = True
    gravity_dataset: GravityDatasetOtfConfig
    model_path: Optional[str] = None


class SegnnNBodyDataLoaderConfig(BaseConfig):
    name: Literal["segnn_nbody"] = "segnn_nbody"
    num_neighbors: int
    gravity_dataset: GravityDatasetOtfConfig
    batch_size: int = 128
    dataset_name: str = "nbody_small"


class EgnnMcNBodyDataLoaderConfig(BaseConfig):
    name: Literal["egnn_mc_nbody"] = "egnn_mc_nbody"
    class_path: str = "nbody_amd.dataloaders.EgnnMcNBodyDataLoader"
    batch_size: int = 128
    num_neighbors: Optional[int] = None
    gravity_dataset: GravityDatasetOtfConfig


class EquiformerV2NBodyDataLoaderConfig(BaseConfig):
    """utils/config_models.py:203-210."""
    name: Literal["equiformer_v2_nbody"] = "equiformer_v2_nbody"
    class_path: str = "nbody_amd.dataloaders.EquiformerV2NBodyDataLoader"
    batch_size: int = 128
    gravity_dataset: GravityDatasetOtfConfig
    max_neighbors: int = 5
    max_radius: float = 4096.0


class ValidationConfig(BaseModel):
    do_validation: bool = False
    split_ratio: float = Field(0.8, ge=0.0, le=1.0)
    validation_frequency: int = 1


class PrecisionMode(str, Enum):
    DOUBLE = "double"
    SINGLE = "single"
    AUTOCAST = "autocast"


class TrainerNBodyConfig(BaseConfig):
    """BaseTrainerConfig + TrainerNBodyConfig (config_models.py:288-366); the trainer
    class itself is outside the native path, the fields feed create_model / run_inference."""
    name: Literal["trainer_nbody"] = "trainer_nbody"
    model_config = {"protected_namespaces": (), "extra": "allow"}
    com_loss: bool = False
    precision_mode: PrecisionMode = PrecisionMode.DOUBLE
    energy_loss: bool = False
    learning_rate: float = 1e-2
    learning_rate_factor: float = 1.0
    learning_rate_warmup_steps: int = 1000
    model_path: Optional[str] = None
    run_name: Optional[str] = None
    save_model_every: int = 10
    test_macros_every: int = 1024
    train_steps: Optional[int] = None
    steps_per_epoch: int = 1
    validation: ValidationConfig = Field(default_factory=ValidationConfig)
    seed: Optional[int] = None
    momentum_loss: bool = False
    momentum_loss_weight: float = 0.0001
    per_atom_loss: bool = False
    self_feed_limit_steps: Optional[int] = None


class MainConfig(BaseModel):
    model_type: str
    dataloader_type: str
    trainer_type: str
    gpu_id: Union[int, str] = 0
    model_config = {"protected_namespaces": ()}


MODEL_CONFIG_NAMES = {"ponita": PonitaModelConfig, "segnn": SegnnModelConfig, "egnn_mc": EgnnMcModelConfig,
                      "equiformer_v2": EquiformerV2ModelConfig}
DATALOADER_CONFIG_NAMES = {"ponita_nbody": PonitaNBodyDataLoaderConfig, "segnn_nbody": SegnnNBodyDataLoaderConfig,
                           "egnn_mc_nbody": EgnnMcNBodyDataLoaderConfig,
                           "equiformer_v2_nbody": EquiformerV2NBodyDataLoaderConfig}
TRAINER_CONFIG_NAMES = {"trainer_nbody": TrainerNBodyConfig}


def load_config(config_path):
    with open(config_path) as f:
        return yaml.safe_load(f)


def _flatten(d, parent=""):
    out = {}
    for k, v in d.items():
        key = f"{parent}.{k}" if parent else k
        if isinstance(v, dict):
            out.update(_flatten(v, key))
        else:
            out[key] = v
    return out


def _set_path(d, dotted, value):
    keys = dotted.split(".")
    for k in keys[:-1]:
        d = d.setdefault(k, {})
    d[keys[-1]] = value


def parse_args(argv=None):
    """utils/config.py::parse_args -> (args, reconstructed_config)."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--config", default=DEFAULT_CONFIG_PATH)
    pre.add_argument("--model_type")
    pre.add_argument("--dataloader_type")
    pre.add_argument("--trainer_type")
    pre.add_argument("--gpu_id")
    known, rest = pre.parse_known_args(argv)
    config = load_config(known.config)
    main = dict(config["main"])
    for k in ("model_type", "dataloader_type", "trainer_type", "gpu_id"):
        if getattr(known, k) is not None:
            main[k] = getattr(known, k)
    main = MainConfig(**main)
    for name, table in ((main.model_type, MODEL_CONFIG_NAMES), (main.dataloader_type, DATALOADER_CONFIG_NAMES),
                        (main.trainer_type, TRAINER_CONFIG_NAMES)):
        if name not in table:
            raise ValueError(f"'{name}' is not a native N-body plugin (available: {sorted(table)})")
    sections = {"model": dict(config["models"][main.model_type]),
                "dataloader": dict(config["dataloaders"][main.dataloader_type]),
                "trainer": dict(config["trainers"][main.trainer_type])}
    # --section.key[.sub] value overrides
    i = 0
    while i < len(rest):
        tok = rest[i]
        if not tok.startswith("--") or "." not in tok:
            raise SystemExit(f"unrecognised argument {tok!r}")
        if "=" in tok:
            key, val = tok[2:].split("=", 1)
            i += 1
        else:
            key, val = tok[2:], rest[i + 1]
            i += 2
        sec, path = key.split(".", 1)
        if sec not in sections:
            raise SystemExit(f"unknown config section {sec!r}")
        _set_path(sections[sec], path, yaml.safe_load(val))
    validated = {"model": MODEL_CONFIG_NAMES[main.model_type](**sections["model"]),
                 "dataloader": DATALOADER_CONFIG_NAMES[main.dataloader_type](**sections["dataloader"]),
                 "trainer": TRAINER_CONFIG_NAMES[main.trainer_type](**sections["trainer"])}
    flat = {"config": known.config, **main.model_dump()}
    nested = {}
    for sec in ("model", "dataloader", "trainer"):
        d = validated[sec].model_dump(mode="json")
        nested[sec] = SimpleNamespace(class_path=d.pop("class_path"))
        for k, v in _flatten(d).items():
            flat[k.split(".")[-1]] = v
    args = SimpleNamespace(**flat, **nested)
    reconstructed = {"main": main.model_dump(),
                     "models": {main.model_type: validated["model"].model_dump(mode="json")},
                     "dataloaders": {main.dataloader_type: validated["dataloader"].model_dump(mode="json")},
                     "trainers": {main.trainer_type: validated["trainer"].model_dump(mode="json")}}
    return args, reconstructed


def load_class_from_args(args, section: str):
    """utils_train.py:19-24."""
    return import_class(getattr(args, section).class_path)


def create_model(args, train_dataloader=None):
    """utils_train.py:27-137, native families; the class comes from ``model.class_path``
    so a config can point at a subclass."""
    cls = load_class_from_args(args, "model")
    if args.model_type == "segnn":
        if args.dataloader_type not in ("segnn_nbody", "segnn_nbody_offline"):
            raise ValueError(f"Unknown combination of model {args.model_type} and dataloader {args.dataloader_type}")
        return cls(num_layers=args.num_layers, hidden_features=args.hidden_features, lmax_h=args.lmax_h)
    if args.model_type == "ponita":
        return cls(layers=args.num_layers, hidden_dim=args.hidden_features, lr=args.learning_rate)
    if args.model_type == "egnn_mc":
        targets = tuple(args.target.split("+")) if isinstance(getattr(args, "target", None), str) else (
            "pos_dt", "vel")
        hf = getattr(args, "hidden_features", 128)
        from .dataloaders import get_device
        return cls(node_input_dim=getattr(args, "node_input_dim", 2), edge_attr_dim=getattr(args, "edge_attr_dim", 4),
                   hidden_node_dim=getattr(args, "hidden_node_dim", hf),
                   hidden_edge_dim=getattr(args, "hidden_edge_dim", hf),
                   hidden_coord_dim=getattr(args, "hidden_coord_dim", hf), num_layers=getattr(args, "num_layers", 4),
                   target_names=targets, activation=getattr(args, "activation", "silu"),
                   coords_weight=getattr(args, "coords_weight", 1.0), recurrent=getattr(args, "recurrent", True),
                   norm_diff=getattr(args, "norm_diff", False), tanh=getattr(args, "tanh", False),
                   device=get_device(args.gpu_id))
    if args.model_type in ("equiformer", "equiformer_v2"):   # utils_train.py:30-54
        from .dataloaders import get_device
        return cls(device=get_device(args.gpu_id), use_pbc=args.use_pbc, max_neighbors=args.max_neighbors,
                   max_radius=args.max_radius, num_layers=args.num_layers,
                   attn_hidden_channels=args.attn_hidden_channels, sphere_channels=args.sphere_channels,
                   num_heads=args.num_heads, attn_alpha_channels=args.attn_alpha_channels,
                   attn_value_channels=args.attn_value_channels, ffn_hidden_channels=args.ffn_hidden_channels,
                   lmax_list=args.lmax_list, mmax_list=args.mmax_list, grid_resolution=args.grid_resolution,
                   edge_channels=args.edge_channels, use_atom_edge_embedding=args.use_atom_edge_embedding,
                   share_atom_edge_embedding=args.share_atom_edge_embedding,
                   distance_function=args.distance_function, num_distance_basis=args.num_distance_basis,
                   attn_activation=args.attn_activation, use_s2_act_attn=args.use_s2_act_attn,
                   ffn_activation=args.ffn_activation)
    raise ValueError(f"Unknown model {args.model_type}")
