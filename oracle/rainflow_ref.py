"""ORACLE (test infrastructure only): scalar restatement of rainflow cycle counting as DER-VET's battery degradation
uses it (`rainflow==3.0.0`, `requirements.txt:22`; storagevet's BatteryTech degradation calls it on the window's SOE
profile -- storagevet is absent from the reference snapshot, so the caller is restated in
der-vet_amd/dervet_hip/degradation.py and its parity is UNPINNED).

The algorithm is ASTM E1049-85 section 5.4.4 (rainflow counting) in the form of that package:
  1. reversals: the first point, every point where the series changes direction (runs of equal values
     collapsed), and the last point;
  2. three-point stack: push each reversal; while the stack holds >= 3 points, with X = |s[-1] - s[-2]| and
     Y = |s[-2] - s[-3]|: stop if X < Y; if the stack holds exactly 3 points, Y contains the starting point: count it
     as a half cycle and drop the first point; otherwise count Y as a full cycle and remove its two points;
  3. the ranges left on the stack are half cycles.
Pinned by the standard's worked example (ASTM E1049-85 Fig. 6 / X1.4: loads -2, 1, -3, 5, -1, 3, -4, 4, -2 give
ranges 3: 0.5, 4: 1.5, 6: 0.5, 8: 1.0, 9: 0.5; tests/test_degradation.py).
"""


def reversals(series):
    """Indices of the reversal points (first, turning points, last)."""
    x = list(series)
    if len(x) < 2:
        return list(range(len(x)))
    out = [0]
    d_last = x[1] - x[0]
    last = 1
    for i in range(2, len(x)):
        if x[i] == x[last]:
            continue
        d = x[i] - x[last]
        if d_last * d < 0:
            out.append(last)
        d_last = d
        last = i
    out.append(len(x) - 1)
    return out


def cycles(series):
    """[(range, count)] in extraction order (count 0.5 or 1.0)."""
    x = list(series)
    if len(x) < 2:
        return []
    pts = [x[i] for i in reversals(x)]
    stack, out = [], []
    for p in pts:
        stack.append(p)
        while len(stack) >= 3:
            X = abs(stack[-1] - stack[-2])
            Y = abs(stack[-2] - stack[-3])
            if X < Y:
                break
            if len(stack) == 3:
                out.append((Y, 0.5))
                stack.pop(0)
            else:
                out.append((Y, 1.0))
                last = stack.pop()
                stack.pop()
                stack.pop()
                stack.append(last)
    for a, b in zip(stack[:-1], stack[1:]):
        out.append((abs(b - a), 0.5))
    return out


def count_cycles(series):
    """{range: total count}, the package's count_cycles without binning."""
    acc = {}
    for r, c in cycles(series):
        acc[r] = acc.get(r, 0.0) + c
    return sorted(acc.items())
