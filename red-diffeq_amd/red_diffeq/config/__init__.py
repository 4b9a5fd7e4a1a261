from .config_dict import ConfigDict
from .config_utils import load_config, print_config, save_config, update_config
from .default_config import get_config, get_marmousi_config

__all__ = ["ConfigDict", "get_config", "get_marmousi_config", "load_config", "save_config", "update_config",
           "print_config"]
