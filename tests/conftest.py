"""Test configuration: `gpu` marker, import paths.

Paths: the repo root (bench/__graft_entry__), ar-nerf_amd/ (the product's
reference-shaped modules: vren, models.*, losses) and oracle/ (the checker).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ar-nerf_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libngp_amd.so on cuda:0)")
