"""Fold TunableOp result files (tools/tune_gemms.sh, one per workload) into one selection file:
the Validator lines of the first file, then every (op, shape) entry once -- a shape tuned in
several runs keeps its fastest measurement.

    python tools/merge_tuning.py OUT.csv IN1.csv [IN2.csv ...]
"""
import sys


def main(out, inputs):
    head, best = [], {}
    for i, path in enumerate(inputs):
        for line in open(path):
            f = line.rstrip("\n").split(",")
            if f[0] == "Validator":
                if i == 0:
                    head.append(line.rstrip("\n"))
                continue
            if len(f) < 4:
                continue
            key, t = (f[0], f[1]), float(f[3])
            if key not in best or t < best[key][0]:
                best[key] = (t, line.rstrip("\n"))
    with open(out, "w") as fo:
        fo.write("\n".join(head + [v[1] for v in best.values()]) + "\n")
    print(f"{out}: {len(best)} entries from {len(inputs)} files")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
