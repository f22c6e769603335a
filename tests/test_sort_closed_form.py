"""The claim re-sort's wave-parallel Hoare passes (ks_solve.hip w_partition / w_partition_equal / w_hoare)
rest on a closed form of Go 1.21's partition_func and partitionEqual_func (src/sort/zsortfunc.go, the
sort.Slice that scheduler.go:247 calls): the boundary is a + #(key < pivot) (a + 1 + #(key <= pivot)), and
the i/j scans exchange the k-th wrong-side entry of the left region with the k-th wrong-side entry of the
right region counted from the right end.  Checked here against the loops themselves on random ranges with
many ties (the claims' pod counts tie heavily), payloads included, so the tie order is compared too."""
import random


def go_partition(d, a, b, pivot):
    d[a], d[pivot] = d[pivot], d[a]
    i, j = a + 1, b - 1
    while i <= j and d[i][0] < d[a][0]:
        i += 1
    while i <= j and not d[j][0] < d[a][0]:
        j -= 1
    if i > j:
        d[j], d[a] = d[a], d[j]
        return j, True
    d[i], d[j] = d[j], d[i]
    i, j = i + 1, j - 1
    while True:
        while i <= j and d[i][0] < d[a][0]:
            i += 1
        while i <= j and not d[j][0] < d[a][0]:
            j -= 1
        if i > j:
            break
        d[i], d[j] = d[j], d[i]
        i, j = i + 1, j - 1
    d[j], d[a] = d[a], d[j]
    return j, False


def go_partition_equal(d, a, b, pivot):
    d[a], d[pivot] = d[pivot], d[a]
    i, j = a + 1, b - 1
    while True:
        while i <= j and not d[a][0] < d[i][0]:
            i += 1
        while i <= j and d[a][0] < d[j][0]:
            j -= 1
        if i > j:
            break
        d[i], d[j] = d[j], d[i]
        i, j = i + 1, j - 1
    return i


def closed_hoare(d, l0, m, r1, bad_left, bad_right):
    left = [p for p in range(l0, m) if bad_left(d[p][0])]
    right = [p for p in range(r1 - 1, m - 1, -1) if bad_right(d[p][0])]
    assert len(left) == len(right)
    for x, y in zip(left, right):
        d[x], d[y] = d[y], d[x]
    return len(left)


def closed_partition(d, a, b, pivot):
    d[a], d[pivot] = d[pivot], d[a]
    pk = d[a][0]
    j = a + sum(1 for p in range(a + 1, b) if d[p][0] < pk)
    k = closed_hoare(d, a + 1, j + 1, b, lambda x: x >= pk, lambda x: x < pk)
    d[j], d[a] = d[a], d[j]
    return j, k == 0


def closed_partition_equal(d, a, b, pivot):
    d[a], d[pivot] = d[pivot], d[a]
    pk = d[a][0]
    m = a + 1 + sum(1 for p in range(a + 1, b) if d[p][0] <= pk)
    closed_hoare(d, a + 1, m, b, lambda x: x > pk, lambda x: x <= pk)
    return m


def test_hoare_closed_form_matches_go_loops():
    rng = random.Random(1)
    for _ in range(6000):
        n = rng.randint(1, 90)
        a = rng.randint(0, n - 1)
        b = rng.randint(a + 1, n)
        keys = [rng.randint(0, rng.randint(1, 8)) for _ in range(n)]
        if rng.random() < 0.5:  # nearly sorted, as after one placement
            keys.sort()
            k = rng.randrange(n)
            keys[k] += 1
        base = [(x, i) for i, x in enumerate(keys)]
        pivot = rng.randint(a, b - 1)
        d1, d2 = list(base), list(base)
        assert go_partition(d1, a, b, pivot) == closed_partition(d2, a, b, pivot)
        assert d1 == d2
        d1, d2 = list(base), list(base)
        assert go_partition_equal(d1, a, b, pivot) == closed_partition_equal(d2, a, b, pivot)
        assert d1 == d2
