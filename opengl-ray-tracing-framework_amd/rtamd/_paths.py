"""Filesystem locations of the in-tree libraries, assets and fixtures."""
from __future__ import annotations

import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent.parent          # opengl-ray-tracing-framework_amd/
REPO_ROOT = PKG_DIR.parent
LIB_DIR = PKG_DIR / "lib"
ASSET_DIR = REPO_ROOT / "assets"
ORACLE_DIR = REPO_ROOT / "oracle"
GOLDEN_DIR = REPO_ROOT / "tests" / "golden"
REFERENCE_DIR = Path(os.environ.get("RT_REFERENCE_DIR", "/root/reference"))


def lib_path(name: str) -> Path:
    p = LIB_DIR / name
    if not p.exists():
        raise FileNotFoundError(f"{p} not built: run `make -C {PKG_DIR}` (or __graft_entry__.build())")
    return p
