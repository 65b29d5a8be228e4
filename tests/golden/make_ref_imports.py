"""Writes tests/golden/ref_imports.json: every `from nets... / from utils...`
name that the reference's callers (predict.py and every train_*.py under
/root/reference/JABD2080ti) import.  The reference is parsed as text with
`ast` — never imported or run.  Run here (the reference is absent on the GPU
box); the JSON is the committed fixture tests/test_dropin.py checks."""
import ast
import glob
import json
import os

REF = "/root/reference/JABD2080ti"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_imports.json")


def main():
    names = {}
    files = sorted(glob.glob(os.path.join(REF, "train_*.py"))) + [os.path.join(REF, "predict.py")]
    for path in files:
        tree = ast.parse(open(path, encoding="utf-8", errors="replace").read())
        for node in ast.walk(tree):
            if isinstance(node, ast.ImportFrom) and node.module and \
                    node.module.split(".")[0] in ("nets", "utils"):
                for a in node.names:
                    key = f"{node.module}:{a.name}"
                    names.setdefault(key, []).append(f"{os.path.basename(path)}:{node.lineno}")
    with open(OUT, "w") as f:
        json.dump(dict(sorted(names.items())), f, indent=1)
    print(f"{len(names)} names -> {OUT}")


if __name__ == "__main__":
    main()
