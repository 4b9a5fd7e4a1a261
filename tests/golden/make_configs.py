"""Fixture generator (run in the build container, where /root/reference exists): the reference's own
YAML configs parsed with PyYAML's SafeLoader and stored as JSON data under tests/golden/configs/
(the parsed values, not the YAML text).  tests/test_gpu_script.py writes each back out as a config
file and runs scripts/run_inversion.py's main() on it unchanged.
python tests/golden/make_configs.py"""
import json
import os

import yaml

REF = "/root/reference/configs"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")
NAMES = {"default": "default.yaml", "openfwi_red-diffeq": "openfwi/red-diffeq.yaml",
         "marmousi_red-diffeq": "marmousi/red-diffeq.yaml"}

if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    for name, rel in NAMES.items():
        with open(os.path.join(REF, rel)) as f:
            cfg = yaml.safe_load(f)
        with open(os.path.join(OUT, name + ".json"), "w") as f:
            json.dump({"source": f"configs/{rel}", "config": cfg}, f, indent=1, sort_keys=True)
        print(name, sorted(cfg))
