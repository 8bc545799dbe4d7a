"""Per-chunk kernel timeline of a rocprofv3 kernel trace of the cascade bench.
usage: python chunk_timeline.py TRACE.csv [chunks]"""
import csv
import sys

NAMES = [('void ', ''), ('Shape<1, 7, 2, 2, 2, 1, 28, 2>', 'VAD'), ('Shape<1, 16, 4, 4, 4, 1, 64, 2>', 'KWS'),
         ('Shape<2, 18, 5, 5, 5, 3, 72, 41>', 'S2I'), ('(anonymous namespace)::', '')]


def short(n):
    n = n.split('(')[0]
    for a, b in NAMES:
        n = n.replace(a, b)
    return n


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    begins = [i for i, r in enumerate(rows) if 'casc_begin' in r['Kernel_Name']]
    for bi in begins[-k - 1:-1]:
        t0 = int(rows[bi]['Start_Timestamp'])
        end = next((b for b in begins if b > bi), len(rows))
        print('--- chunk')
        for r in rows[max(0, bi - 2):end]:
            s = (int(r['Start_Timestamp']) - t0) / 1e3
            e = (int(r['End_Timestamp']) - t0) / 1e3
            print(f"{short(r['Kernel_Name'])[:48]:48s} {s:8.1f} {e:8.1f} {e - s:7.1f}  grid {r['Grid_Size_X']} wg {r['Workgroup_Size_X']}")


if __name__ == '__main__':
    main()
