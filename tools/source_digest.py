"""The library's source digest: SHA-1 over the files compiled into it —
csrc/*.hip, *.cpp, *.hpp and the public headers include/*.h, *.hpp — each as
its path relative to the repo root, NUL, content, in sorted path order
(bench.py imports this function).

  python3 tools/source_digest.py            print it
  python3 tools/source_digest.py OUT.h      write `#define CSM_SOURCE_DIGEST "..."`
                                            to OUT.h when it changed (Makefile)
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCE_DIRS = ((os.path.join("roborts-edu-slam_amd", "csrc"), (".hip", ".cpp", ".hpp")),
               ("include", (".h", ".hpp")))


def digest(root: str = ROOT) -> str:
    files = []
    for d, exts in SOURCE_DIRS:
        files += [os.path.join(d, f) for f in os.listdir(os.path.join(root, d)) if f.endswith(exts)]
    h = hashlib.sha1()
    for rel in sorted(files):
        with open(os.path.join(root, rel), "rb") as fh:
            h.update(rel.encode() + b"\0" + fh.read())
    return h.hexdigest()[:12]


if __name__ == "__main__":
    d = digest()
    if len(sys.argv) < 2:
        print(d)
        sys.exit(0)
    text = f'#define CSM_SOURCE_DIGEST "{d}"\n'
    out = sys.argv[1]
    if not os.path.exists(out) or open(out).read() != text:
        os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
        with open(out, "w") as fh:
            fh.write(text)
