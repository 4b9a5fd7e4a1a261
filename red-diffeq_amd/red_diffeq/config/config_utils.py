"""YAML config I/O (reference red_diffeq/config/config_utils.py:6-53)."""
from pathlib import Path
from typing import Union

import yaml

from .config_dict import ConfigDict


def load_config(config_path: Union[str, Path]) -> ConfigDict:
    config_path = Path(config_path)
    if not config_path.exists():
        raise FileNotFoundError(f"Config file not found: {config_path}")
    with open(config_path, "r") as f:
        d = yaml.safe_load(f)
    return ConfigDict(d or {})


def _tuples_to_lists(o):
    if isinstance(o, dict):
        return {k: _tuples_to_lists(v) for k, v in o.items()}
    if isinstance(o, (tuple, list)):
        return [_tuples_to_lists(v) for v in o]
    return o


def save_config(config: ConfigDict, output_path: Union[str, Path]) -> None:
    output_path = Path(output_path)
    output_path.parent.mkdir(parents=True, exist_ok=True)
    with open(output_path, "w") as f:
        yaml.dump(_tuples_to_lists(config.to_dict()), f, default_flow_style=False, sort_keys=False)


def update_config(config: ConfigDict, **kwargs) -> ConfigDict:
    for k, v in kwargs.items():
        if not hasattr(config, k):
            print(f"Warning: '{k}' not in config, adding it")
        setattr(config, k, v)
    return config


def print_config(config: ConfigDict, prefix: str = "") -> None:
    if not prefix:
        print("=" * 60 + "\nConfiguration:\n" + "=" * 60)
    for k, v in sorted(config.items()):
        if isinstance(v, ConfigDict):
            print(f"{prefix}{k}:")
            print_config(v, prefix=prefix + "  ")
        else:
            print(f"{prefix}{k}: {v}")
    if not prefix:
        print("=" * 60)
