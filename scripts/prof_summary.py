"""Summarise a rocprofv3 kernel_stats.csv into a markdown table (top kernels by total time)."""
import csv
import sys


def main(path, top=20):
    rows = list(csv.DictReader(open(path)))
    print("| total ms | calls | avg us | max us | % | kernel |")
    print("|---:|---:|---:|---:|---:|---|")
    for r in rows[:top]:
        name = r["Name"].replace("(anonymous namespace)::", "").replace("|", "/")
        if len(name) > 110:
            name = name[:110] + "..."
        print(f"| {float(r['TotalDurationNs'])/1e6:.2f} | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
              f"{float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} | `{name}` |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
