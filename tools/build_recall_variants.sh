#!/bin/bash
# Builds k_score_filter A/B variants of liblgcn.so into tools/_variants/ (see tools/recall_variants.py).
# The variants are not in the product source: each is spliced into a copy of lgcn_recall.hip here
# (NO_MFMA: the MFMA chain replaced by one multiply per accumulator; NO_EPI: the epilogue skipped).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/movie-recommender-system-with-gnns_amd/csrc
T=$R/tools/_variants
mkdir -p "$T/src"
cp "$C"/*.hip "$C"/*.cpp "$C"/*.h "$T/src/"
python3 - "$T/src/lgcn_recall.hip" <<'EOF'
import sys
p = sys.argv[1]
s = open(p).read()
mfma = "        constexpr int G = (H / 4) >= 4 ? 4 : (H / 4);\n"
epi = "        // epilogue: column = candidate j (this lane's), rows = queries; branch-free test, and\n"
assert mfma in s and epi in s
s = s.replace(mfma, mfma + """#ifdef LGCN_VARIANT_NO_MFMA
        for (int r = 0; r < 16; ++r) acc[r] = brow[r] * a[r];
        if (false)
#endif
""", 1)
s = s.replace(epi, """#ifdef LGCN_VARIANT_NO_EPI
        if (acc[0] == 12345.f && acc[15] == 54321.f) list_n[0] = 1;  // keep acc live; never true
        if (nxt < nblk) land(buf ^ 1);
        __syncthreads();
        buf ^= 1;
        continue;
#endif
""" + epi, 1)
open(p, "w").write(s)
EOF
# the tree's provenance hash (as tools/build_variant.py links it), so lgcn_amd._ffi loads the variant
SHA=$(cd "$R" && python3 -c "import __graft_entry__ as g; print(g._ffi_module().source_sha256())")
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -ffp-contract=off -I$R/include -DLGCN_SOURCE_SHA256=$SHA"
SRC=$(ls "$T"/src/*.hip "$T"/src/*.cpp)
for v in "$@"; do
  /opt/rocm/bin/hipcc $F -DLGCN_VARIANT_$v $SRC -o "$T/$v.so" &
done
wait
