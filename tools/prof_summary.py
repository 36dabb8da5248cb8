"""Summarise a rocprofv3 kernel_stats.csv into a markdown table."""
import csv
import sys


def main(path, title, out=None, top=25):
    rows = list(csv.DictReader(open(path)))
    lines = ['# ' + title, '',
             '| kernel | calls | total us | avg us | % |',
             '|---|---|---|---|---|']
    for r in rows[:top]:
        lines.append('| `%s` | %s | %.1f | %.1f | %.1f |' % (
            r['Name'][:80], r['Calls'], float(r['TotalDurationNs']) / 1e3,
            float(r['AverageNs']) / 1e3, float(r['Percentage'])))
    txt = '\n'.join(lines) + '\n'
    if out:
        open(out, 'w').write(txt)
    print(txt)


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
