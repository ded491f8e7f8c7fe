#!/bin/bash
# Build an A/B library from a transformed copy of the sources: exp/v_<name>/ holds a copy of
# csrc/ (+ include/) with `python <transform.py> <file>` applied to each listed file, built with
# the product Makefile; prints the library path (exp/v_<name>/real-time-voice-cloning_amd/
# wavernn_amd/libwavernn_mi355x.so, loaded with WRNN_LIB=...).
# Usage: tools/build_patched.sh <name> <transform.py> file.hip [file.hip ...]
set -eu
name=$1 tr=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
v=$root/exp/v_$name
rm -rf "$v"
mkdir -p "$v/real-time-voice-cloning_amd/wavernn_amd"
cp -r "$root/include" "$v/include"
cp -r "$root/real-time-voice-cloning_amd/csrc" "$v/real-time-voice-cloning_amd/csrc"
rm -rf "$v/real-time-voice-cloning_amd/csrc/build"
for f in "$@"; do python3 "$root/$tr" "$v/real-time-voice-cloning_amd/csrc/$f"; done
make -C "$v/real-time-voice-cloning_amd/csrc" -j8 > "$v/build.log" 2>&1 || { tail -30 "$v/build.log"; exit 1; }
echo "$v/real-time-voice-cloning_amd/wavernn_amd/libwavernn_mi355x.so"
