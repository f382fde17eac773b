"""Build an A/B variant of liblgcn.so: the tree's objects, with ONE source recompiled under extra
-D flags, linked (with the same provenance hash — the sources are the tree's) into another path.
On the GPU box, copy it over lgcn_amd/liblgcn.so between two bench runs (the box's tree is a
scratch copy).

python tools/build_variant.py OUT.so SOURCE.hip -DNAME=VALUE [...]
python tools/build_variant.py OUT.so SOURCE.hip=OTHER_FILE.hip   (SOURCE's translation unit from another file,
                                                             e.g. the last commit's: git show HEAD:... > ab/x.hip)"""
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import __graft_entry__ as G  # noqa: E402


def main():
    out, src, defs = pathlib.Path(sys.argv[1]).resolve(), sys.argv[2], sys.argv[3:]
    src, _, other = src.partition("=")
    src_path = pathlib.Path(other).resolve() if other else G.CSRC / src
    G.build()  # the tree's objects up to date
    hipcc = "/opt/rocm/bin/hipcc"
    flags = [f for f in G.HIPCC_FLAGS if f != "-shared"]
    objdir = G.PKG / "build"
    var_obj = objdir / f"variant_{src}.o"
    subprocess.run([hipcc, *flags, *defs, f"-I{G.ROOT / 'include'}", "-I" + str(G.CSRC), "-c", str(src_path), "-o", str(var_obj)],
                   check=True)
    ffi = G._ffi_module()
    objs = [var_obj if s == src else objdir / (s + ".o") for s in ffi.SOURCES] + [objdir / "lgcn_build.cpp.o"]
    out.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run([hipcc, "--offload-arch=gfx950", "-fPIC", "-shared", *map(str, objs), "-o", str(out)], check=True)
    print(f"{out}: {src} from {src_path} with {' '.join(defs)}")


if __name__ == "__main__":
    main()
