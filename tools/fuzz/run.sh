#!/bin/bash
# CPU-only: build the host decoder with ASan+UBSan and fuzz it on baseline,
# progressive and multi-scan files (tools/fuzz/make_inputs.py).
set -eu
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${TMPDIR:-/tmp}/hjd_fuzz
mkdir -p $O
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer \
    -I$R/include -I$R/ocljpegdecoder_amd/csrc $R/ocljpegdecoder_amd/csrc/jpeg_host.cpp $R/tools/fuzz/host_decode_fuzz.cpp \
    -o $O/fuzz -lpthread
PYTHONPATH=$R:$R/tests python3 $R/tools/fuzz/make_inputs.py $O
$O/fuzz ${1:-2000} $O/*.jpg
