"""Running the Node-API addon (bindings/napi) from the tests: build it if needed, run a node
script against it, read back its JSON. Test infrastructure."""
from __future__ import annotations

import json
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADDON_DIR = os.path.join(ROOT, "bindings", "napi")
ADDON = os.path.join(ADDON_DIR, "build", "thesia.node")


def node_bin():
    return shutil.which("node")


def ensure_addon() -> str:
    """The built addon's path (make -C bindings/napi when it is missing or older than its source)."""
    src = os.path.join(ADDON_DIR, "thesia_napi.cc")
    if not os.path.exists(ADDON) or os.path.getmtime(ADDON) < os.path.getmtime(src):
        subprocess.run(["make", "-C", ADDON_DIR], check=True, capture_output=True, timeout=300)
    return ADDON


def run_node(script: str, timeout: int = 120) -> dict:
    """Run `script` with `t` bound to the addon; the script prints one JSON object last."""
    prog = f"const t = require({json.dumps(ensure_addon())});\n" + script
    r = subprocess.run([node_bin(), "-e", prog], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])
