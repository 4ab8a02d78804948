#!/bin/bash
# build_variant.sh NAME "HIPDEFS" -- a profiling variant of libh264scroll.so
# (e.g. -DSCROLL_ABL_STOP=2) in variants/NAME/ (git-ignored; travels to the
# GPU box with the tree).  Select it with H264SCROLL_LIB=variants/NAME/libh264scroll.so.
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
DEFS=$2
OUT=$HERE/../variants/$NAME
mkdir -p "$OUT/obj"
make -s -C "$HERE" -j8 OBJ="$OUT/obj" LIB="$OUT/libh264scroll.so" HIPDEFS="$DEFS" "$OUT/libh264scroll.so"
