set -u
BENCH_ARGS="--utts-per-gpu 7" bash tools/ab.sh real-time-voice-cloning_amd/wavernn_amd/libwavernn_mi355x.so exp/lib_wspin.so && TAG=_c2 bash tools/ab.sh real-time-voice-cloning_amd/wavernn_amd/libwavernn_mi355x.so exp/lib_pspin.so
