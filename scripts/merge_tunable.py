#!/usr/bin/env python
"""Merge TunableOp result tables: the rows of ``new`` whose (op, shape) key the base table lacks
are appended to ``base`` (the base's rows and validators win).  Writes ``out``.

    python scripts/merge_tunable.py base.csv new.csv out.csv
"""
import sys


def rows(path):
    with open(path) as f:
        return [ln.rstrip("\n") for ln in f if ln.strip()]


def main():
    base, new, out = sys.argv[1:4]
    b = rows(base)
    keys = {tuple(ln.split(",")[:2]) for ln in b if not ln.startswith("Validator")}
    added = [ln for ln in rows(new) if not ln.startswith("Validator") and tuple(ln.split(",")[:2]) not in keys]
    with open(out, "w") as f:
        f.write("\n".join(b + added) + "\n")
    print(f"{len(added)} rows added to {len(b)}")


if __name__ == "__main__":
    main()
