"""Committed golden fixtures: .wv streams + manifest.json (see make_golden.py)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with open(os.path.join(HERE, "manifest.json")) as f:
        man = json.load(f)
    for name, m in sorted(man.items()):
        with open(os.path.join(HERE, m["file"]), "rb") as f:
            yield name, f.read(), m
