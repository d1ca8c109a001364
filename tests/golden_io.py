"""Readers for the golden fixtures written by tests/golden/make_golden.py."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def unpack(d, key, i):
    off = d[key + '_off']
    return d[key][off[i]:off[i + 1]]


def ncases(d, key):
    return len(d[key + '_off']) - 1


def opt(v):
    v = float(v)
    return None if np.isnan(v) else v
