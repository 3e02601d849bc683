"""Go 1.19 ``sort.Slice`` (pdqsort_func, src/sort/zsortfunc.go) for the host facades.

The reference's callers sort with ``sort.Slice``, which is NOT stable: tied elements come
out in an order fixed by pdqsort's pivots, partitions and swaps.  The Go caller of the C
ABI gets that order from Go itself; the Python facades mirror the caller, so they need
the same algorithm (FilterOutSchedulable's priority sort,
CA/core/podlistprocessor/filter_out_schedulable.go:97-99).  The device restates the same
algorithm for Estimate's score sort (estimate.hip k_pdq_*; binpacking_estimator.go:74).
Written from the published Go 1.19 algorithm; the breakPatterns xorshift shifts are
13/17/5 on a uint64 state (the one unpinned assumption).
"""
from __future__ import annotations

from typing import Callable, Sequence


def sort_slice(n: int, less: Callable[[int, int], bool], swap: Callable[[int, int], None]) -> None:
    """sort.Slice over an abstract sequence of length n (Less / Swap by index)."""

    def insertion_sort(a, b):
        for i in range(a + 1, b):
            j = i
            while j > a and less(j, j - 1):
                swap(j, j - 1)
                j -= 1

    def sift_down(lo, hi, first):
        root = lo
        while True:
            child = 2 * root + 1
            if child >= hi:
                return
            if child + 1 < hi and less(first + child, first + child + 1):
                child += 1
            if not less(first + root, first + child):
                return
            swap(first + root, first + child)
            root = child

    def heap_sort(a, b):
        first, lo, hi = a, 0, b - a
        for i in range((hi - 1) // 2, -1, -1):
            sift_down(i, hi, first)
        for i in range(hi - 1, -1, -1):
            swap(first, first + i)
            sift_down(lo, i, first)

    def break_patterns(a, b):
        length = b - a
        if length >= 8:
            r = length
            modulus = 1 << length.bit_length()
            idx = a + (length // 4) * 2 - 1
            for i in range(3):
                r ^= (r << 13) & 0xFFFFFFFFFFFFFFFF
                r ^= r >> 17
                r ^= (r << 5) & 0xFFFFFFFFFFFFFFFF
                other = r & (modulus - 1)
                if other >= length:
                    other -= length
                swap(idx - 1 + i, a + other)

    def choose_pivot(a, b):
        swaps = [0]

        def order2(x, y):
            if less(y, x):
                swaps[0] += 1
                return y, x
            return x, y

        def median(x, y, z):
            x, y = order2(x, y)
            y, z = order2(y, z)
            x, y = order2(x, y)
            return y

        l = b - a
        i, j, k = a + l // 4 * 1, a + l // 4 * 2, a + l // 4 * 3
        if l >= 8:
            if l >= 50:
                i = median(i - 1, i, i + 1)
                j = median(j - 1, j, j + 1)
                k = median(k - 1, k, k + 1)
            j = median(i, j, k)
        hint = 1 if swaps[0] == 0 else (2 if swaps[0] == 12 else 0)     # increasing / decreasing / unknown
        return j, hint

    def partial_insertion_sort(a, b):
        i = a + 1
        for _ in range(5):
            while i < b and not less(i, i - 1):
                i += 1
            if i == b:
                return True
            if b - a < 50:
                return False
            swap(i, i - 1)
            if i - a >= 2:
                j = i - 1
                while j >= 1:
                    if not less(j, j - 1):
                        break
                    swap(j, j - 1)
                    j -= 1
            if b - i >= 2:
                j = i + 1
                while j < b:
                    if not less(j, j - 1):
                        break
                    swap(j, j - 1)
                    j += 1
        return False

    def partition(a, b, pivot):
        swap(a, pivot)
        i, j = a + 1, b - 1
        while i <= j and less(i, a):
            i += 1
        while i <= j and not less(j, a):
            j -= 1
        if i > j:
            swap(j, a)
            return j, True
        swap(i, j)
        i += 1
        j -= 1
        while True:
            while i <= j and less(i, a):
                i += 1
            while i <= j and not less(j, a):
                j -= 1
            if i > j:
                break
            swap(i, j)
            i += 1
            j -= 1
        swap(j, a)
        return j, False

    def partition_equal(a, b, pivot):
        swap(a, pivot)
        i, j = a + 1, b - 1
        while True:
            while i <= j and not less(a, i):
                i += 1
            while i <= j and less(a, j):
                j -= 1
            if i > j:
                break
            swap(i, j)
            i += 1
            j -= 1
        return i

    def pdqsort(a, b, limit):
        was_balanced, was_partitioned = True, True
        while True:
            length = b - a
            if length <= 12:
                insertion_sort(a, b)
                return
            if limit == 0:
                heap_sort(a, b)
                return
            if not was_balanced:
                break_patterns(a, b)
                limit -= 1
            pivot, hint = choose_pivot(a, b)
            if hint == 2:
                i, j = a, b - 1
                while i < j:
                    swap(i, j)
                    i += 1
                    j -= 1
                pivot = (b - 1) - (pivot - a)
                hint = 1
            if was_balanced and was_partitioned and hint == 1:
                if partial_insertion_sort(a, b):
                    return
            if a > 0 and not less(a - 1, pivot):
                a = partition_equal(a, b, pivot)
                continue
            mid, was_partitioned = partition(a, b, pivot)
            left, right = mid - a, b - mid
            threshold = length // 8
            if left < right:
                was_balanced = left >= threshold
                pdqsort(a, mid, limit)
                a = mid + 1
            else:
                was_balanced = right >= threshold
                pdqsort(mid + 1, b, limit)
                b = mid

    pdqsort(0, n, n.bit_length())


def sort_slice_desc(keys: Sequence) -> list:
    """sort.Slice(x, func(i, j) bool { return key(x[i]) > key(x[j]) }): the permutation
    (position k holds input index perm[k])."""
    perm = list(range(len(keys)))
    k = list(keys)

    def less(i, j):
        return k[perm[i]] > k[perm[j]]

    def swap(i, j):
        perm[i], perm[j] = perm[j], perm[i]

    sort_slice(len(perm), less, swap)
    return perm
