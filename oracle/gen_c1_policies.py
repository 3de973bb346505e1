"""Collect the reference's example policies that C1 is built from
(examples/policies/l3/*/*.json and l4/*.json, BASELINE.json configs[0]) into
the fixture tests/golden/c1_policies.json: {relative path: [rules]}.
Test infrastructure: run here, where /root/reference exists; the fixture
(policy data, not code) is what the tests and generators read."""
import glob
import json
import os

REF = "/root/reference/examples/policies"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = {}
    for p in sorted(glob.glob(os.path.join(REF, "l3", "*", "*.json")) +
                    glob.glob(os.path.join(REF, "l4", "*.json"))):
        out[os.path.relpath(p, REF)] = json.load(open(p))
    dst = os.path.join(ROOT, "tests", "golden", "c1_policies.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"{len(out)} policy files -> {dst}")


if __name__ == "__main__":
    main()
