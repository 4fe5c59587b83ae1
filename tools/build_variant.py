"""Build libeggroll from the working tree with extra -D flags into tools/_ab/<name>.so (A/B of compile-time
knobs: EGG_GROUP_M, EGG_PTB_SPLIT, EGG_LA_FOLD ...).  Never loaded by the package; tools/*_lib_ab.py bind it.
usage: python tools/build_variant.py <name> -DKNOB=VALUE [...]"""
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SRCS = ["eggroll_es.hip", "eggroll_lora.hip", "eggroll_model.hip"]


def main(name, flags):
    out = ROOT / "tools" / "_ab" / f"{name}.so"
    out.parent.mkdir(parents=True, exist_ok=True)

    def cc(s):
        o = out.parent / f"{name}_{Path(s).stem}.o"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", *flags,
                        f"-I{ROOT / 'include'}", str(ROOT / "hyperscalees_t2i_amd" / "csrc" / s), "-o", str(o)],
                       check=True, capture_output=True)
        return str(o)
    with ThreadPoolExecutor(3) as ex:
        objs = list(ex.map(cc, SRCS))
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", str(out)], check=True)
    for o in objs:
        Path(o).unlink()
    print(out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
