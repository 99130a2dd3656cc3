"""Config surface of the reference (utils_conf.py:4-42): JSON/YAML load + dotted `--set` overrides.

Accepts config/baseline and config/more_blocks unchanged.  `train.backend` "fsdp"/"deepspeed"
(config/more_blocks:37) map onto this package's data-parallel path (35 M params need no sharding
on a 288 GB part; the reference FSDP path is broken).
"""
from __future__ import annotations

import json
import pathlib


def load_config(path: str) -> dict:
    p = pathlib.Path(path)
    if not p.exists():
        raise FileNotFoundError(f"Config not found: {p}")
    if p.suffix.lower() in (".yml", ".yaml"):
        import yaml
        with p.open() as f:
            return yaml.safe_load(f)
    with p.open() as f:
        return json.load(f)


def parse_value(s: str):
    sl = s.lower()
    if sl in ("true", "false"):
        return sl == "true"
    try:
        return float(s) if "." in s else int(s)
    except ValueError:
        return s


def apply_overrides(cfg: dict, pairs) -> None:
    for pair in pairs:
        if "=" not in pair:
            raise ValueError(f"Invalid override (no '='): {pair}")
        key, val = pair.split("=", 1)
        d = cfg
        parts = key.split(".")
        for k in parts[:-1]:
            if k not in d or not isinstance(d[k], dict):
                d[k] = {}
            d = d[k]
        d[parts[-1]] = parse_value(val)


def dataset_kwargs(cfg: dict) -> dict:
    """train.py:990-1001 mapping of config['dataset'] (crop_hw falsy -> full grid)."""
    ds = cfg["dataset"]
    return dict(K=ds["K"], center=ds["center"], crop_hw=tuple(ds["crop_hw"]) if ds["crop_hw"] else None,
                crop_mode=ds["crop_mode"], time_reverse_p=ds["time_reverse_p"], sample_mode=ds["sample_mode"])
