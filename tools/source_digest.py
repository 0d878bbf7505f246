"""The library's source digest (SHA-1 over csrc/*.hip, *.cpp, *.hpp: name, NUL,
content, in sorted name order; the same as bench.py's source_digest).

  python3 tools/source_digest.py            print it
  python3 tools/source_digest.py OUT.h      write `#define CSM_SOURCE_DIGEST "..."`
                                            to OUT.h when it changed (Makefile)
"""
import hashlib
import os
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "roborts-edu-slam_amd", "csrc")


def digest(csrc: str = CSRC) -> str:
    h = hashlib.sha1()
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".cpp", ".hpp")):
            with open(os.path.join(csrc, f), "rb") as fh:
                h.update(f.encode() + b"\0" + fh.read())
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
