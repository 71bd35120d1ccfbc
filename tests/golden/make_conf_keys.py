"""Generate tests/golden/conf_keys.json: the key set (dotted paths) and the scalar values of
every YAML file under the reference's conf/ (Hydra config surface, conf/config.yaml etc.).

Run in the survey container, where /root/reference exists:
    python tests/golden/make_conf_keys.py
The files are read with yaml.safe_load as data only.  The output is committed; the tests
(tests/test_host_logic.py::test_conf_surface_matches_reference) read only the JSON.
"""
import json
import os

import yaml

REF = "/root/reference/conf"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "conf_keys.json")


def flatten(d, prefix=""):
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(flatten(v, key + "."))
        else:
            out[key] = v
    return out


def main():
    files = {}
    for root, _, names in os.walk(REF):
        for n in sorted(names):
            if not n.endswith(".yaml"):
                continue
            path = os.path.join(root, n)
            with open(path) as f:
                data = yaml.safe_load(f) or {}
            rel = os.path.relpath(path, REF)
            flat = flatten(data)
            files[rel] = {k: (v if isinstance(v, (str, int, float, bool)) or v is None else
                              json.loads(json.dumps(v))) for k, v in sorted(flat.items())}
    with open(OUT, "w") as f:
        json.dump(dict(sorted(files.items())), f, indent=1, sort_keys=True)
    print("wrote", OUT, len(files), "files")


if __name__ == "__main__":
    main()
