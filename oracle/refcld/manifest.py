"""TEST INFRASTRUCTURE.  Provenance of oracle/_ref/librefcld2.so: written by
oracle/refcld/Makefile right after linking, read by refcld.verify_build() on
the GPU box (where /root/reference does not exist) so the reference checks
run only against a binary built from this tree's recipe.

    manifest.py OUT_JSON LIB RECIPE_FILE... -- REFERENCE_SOURCE...

Records sha256 of the library, of each recipe file (refcld.cc, the Makefile:
repo-relative paths, re-hashed on the box) and of each reference source it
was compiled from (recorded only: they do not travel)."""
import hashlib
import json
import os
import sys


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def main():
    out, lib, rest = sys.argv[1], sys.argv[2], sys.argv[3:]
    cut = rest.index("--")
    recipe, sources = rest[:cut], rest[cut + 1:]
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    m = {"library": {"path": os.path.relpath(os.path.abspath(lib), root), "sha256": sha(lib)},
         "recipe": {os.path.relpath(os.path.abspath(p), root): sha(p) for p in recipe},
         "reference_sources": {os.path.basename(p): sha(p) for p in sources}}
    with open(out, "w") as f:
        json.dump(m, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
