#!/bin/bash
# Diagnostic builds of libkoordgpu (separate object dirs): libkoordgpu_diag.so (-DKS_COMMIT_STAMPS, per-phase
# cycles of the general commit kernel), libkoordgpu_cat.so (-DKS_COMMIT_CAT, per-pod-category commit cycles) and
# libkoordgpu_seg.so (-DKS_COMMIT_SEG, the monotone commit kernel's fast-pod iteration split) and
# libkoordgpu_split.so (-DKS_SLOT_SPLIT, the slot evaluation's parts).  Used by
# tools/diag_commit.py; none of them is loaded by the tests, smoke() or bench.py.
set -e
cd "$(dirname "$0")/../koordinator_amd/csrc"
R=$(cd ../.. && pwd)
make -j8 OUT=$R/koordinator_amd/libkoordgpu_diag.so OBJ=$R/build/obj_diag EXTRA_HIPFLAGS=-DKS_COMMIT_STAMPS >/dev/null
make -j8 OUT=$R/koordinator_amd/libkoordgpu_cat.so OBJ=$R/build/obj_cat EXTRA_HIPFLAGS=-DKS_COMMIT_CAT >/dev/null
make -j8 OUT=$R/koordinator_amd/libkoordgpu_seg.so OBJ=$R/build/obj_seg EXTRA_HIPFLAGS=-DKS_COMMIT_SEG >/dev/null
make -j8 OUT=$R/koordinator_amd/libkoordgpu_split.so OBJ=$R/build/obj_split EXTRA_HIPFLAGS="-DKS_COMMIT_STAMPS -DKS_SLOT_SPLIT" >/dev/null
