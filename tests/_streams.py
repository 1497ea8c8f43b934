"""Synthetic stream fixtures: regenerate each stream with tools/_build/h264gen and check it against
the recorded sha256 in tests/golden/synthetic.json (so a drifting generator is caught first)."""
import hashlib
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "tools", "_build", "h264gen")
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "synthetic.json")))
_cache = {}


def stream(name, tmpdir="/tmp"):
    if name in _cache:
        return _cache[name]
    g = GOLDEN[name]
    out = os.path.join(tmpdir, f"m2dec_{name}_{os.getpid()}.264")
    subprocess.run([GEN, "--preset", g["preset"], "--seed", str(g["seed"]), "--frames", str(g["frames"]), "-o", out],
                   check=True, stderr=subprocess.DEVNULL)
    data = open(out, "rb").read()
    os.unlink(out)
    assert hashlib.sha256(data).hexdigest() == g["sha256"], f"generator output drifted for {name}"
    _cache[name] = data
    return data
