#!/bin/bash
# CPU-only: build the GPU entropy decoder's host emulation (hjd_entropy.hip and
# what it links against) with host-side AddressSanitizer + UBSan, and fuzz it
# on damaged sequential JPEGs, one scan or several (tools/fuzz/entropy_emulate_fuzz.cpp).
set -eu
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${TMPDIR:-/tmp}/hjd_efuzz
mkdir -p $O
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
FLAGS="-std=c++17 -O1 -g -fno-omit-frame-pointer -I$R/include -I$R/ocljpegdecoder_amd/csrc"
C=$R/ocljpegdecoder_amd/csrc
pids=()
newest_hdr=$(ls -t $C/*.hpp $C/*.h $R/include/*.h | head -1)
for f in hjd_entropy hjd_runtime idct_compat stream_pipeline numa_affinity hjd_probe; do
  [ $O/$f.o -nt $C/$f.hip ] && [ $O/$f.o -nt $newest_hdr ] || { /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $SAN -c $C/$f.hip -o $O/$f.o & pids+=($!); }
done
[ $O/jpeg_host.o -nt $C/jpeg_host.cpp ] && [ $O/jpeg_host.o -nt $newest_hdr ] || { /opt/rocm/bin/hipcc -x c++ $FLAGS $SAN -c $C/jpeg_host.cpp -o $O/jpeg_host.o & pids+=($!); }
for p in ${pids[@]+"${pids[@]}"}; do wait $p; done
/opt/rocm/bin/hipcc -x c++ $FLAGS $SAN -c $R/tools/fuzz/entropy_emulate_fuzz.cpp -o $O/main.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=address,undefined -fno-gpu-sanitize $O/*.o -o $O/efuzz -lpthread
PYTHONPATH=$R:$R/tests python3 $R/tools/fuzz/make_inputs.py $O >/dev/null
# larger seeds: many subsequences and several sync groups per frame at small S
python3 - $O <<'PY'
import io, sys
import numpy as np
from PIL import Image
rng = np.random.default_rng(11)
for name, (w, h, q, sub, kw) in {"big420": (512, 384, 90, 2, {}), "big444dri": (320, 240, 95, 0, {"restart_marker_blocks": 5}),
                                 "big422": (400, 200, 75, 1, {})}.items():
    x = np.linspace(0, 255, w)[None, :, None] + rng.normal(0, 20, (h, w, 3))
    b = io.BytesIO()
    Image.fromarray(np.clip(x, 0, 255).astype(np.uint8)).save(b, format="JPEG", quality=q, subsampling=sub, **kw)
    open(f"{sys.argv[1]}/{name}.jpg", "wb").write(b.getvalue())
PY
$O/efuzz ${1:-200} $O/*.jpg
