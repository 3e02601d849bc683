/*
 * gosort.c — restatement of Go 1.19 sort.Slice (pattern-defeating quicksort,
 * src/sort/zsortfunc.go pdqsort_func and src/sort/sort.go xorshift / nextPowerOfTwo /
 * Slice).  TEST INFRASTRUCTURE ONLY (the checker of the device sort).
 *
 * The reference sorts with sort.Slice (CA/estimator/binpacking_estimator.go:74, score
 * descending; CA/core/podlistprocessor/filter_out_schedulable.go:97-99, priority
 * descending) and is built with Go 1.19 (/root/reference/builder/Dockerfile:15,
 * CA/go.mod:3).  sort.Slice is not stable: the order of tied elements is determined by
 * pdqsort's pivots, partitions and swaps, so parity of the pod order (the scheduled pods
 * Estimate returns, the FilterOutSchedulable processing order) needs the same algorithm.
 * The Go standard library is not in this container; this is
 * written from the published algorithm of Go 1.19's sort package, operation for
 * operation: the same comparisons (Less) and the same swaps (Swap) in the same order.
 *
 * Here less(i, j) = key[i] > key[j] (both reference sorts are descending on one key);
 * the elements are (key, original index) pairs and the result is the permutation.
 */
#include <stdint.h>
#include <stdlib.h>

typedef struct gs_elem { double key; int32_t idx; } gs_elem;

static int64_t gs_break_calls, gs_heap_calls;         /* breakPatterns / heapSort calls so far */
void go_sort_stats(int64_t* out2) { out2[0] = gs_break_calls; out2[1] = gs_heap_calls; }

static int gs_less(const gs_elem* d, int64_t i, int64_t j) { return d[i].key > d[j].key; }
static void gs_swap(gs_elem* d, int64_t i, int64_t j) { gs_elem t = d[i]; d[i] = d[j]; d[j] = t; }

enum { unknownHint = 0, increasingHint = 1, decreasingHint = 2 };

/* insertionSort_func */
static void insertion_sort(gs_elem* d, int64_t a, int64_t b) {
    for (int64_t i = a + 1; i < b; i++)
        for (int64_t j = i; j > a && gs_less(d, j, j - 1); j--) gs_swap(d, j, j - 1);
}

/* siftDown_func */
static void sift_down(gs_elem* d, int64_t lo, int64_t hi, int64_t first) {
    int64_t root = lo;
    for (;;) {
        int64_t child = 2 * root + 1;
        if (child >= hi) return;
        if (child + 1 < hi && gs_less(d, first + child, first + child + 1)) child++;
        if (!gs_less(d, first + root, first + child)) return;
        gs_swap(d, first + root, first + child);
        root = child;
    }
}

/* heapSort_func */
static void heap_sort(gs_elem* d, int64_t a, int64_t b) {
    gs_heap_calls++;
    int64_t first = a, lo = 0, hi = b - a;
    for (int64_t i = (hi - 1) / 2; i >= 0; i--) sift_down(d, i, hi, first);
    for (int64_t i = hi - 1; i >= 0; i--) {
        gs_swap(d, first, first + i);
        sift_down(d, lo, i, first);
    }
}

/* bits.Len(uint(x)) */
static int bits_len(uint64_t x) { int n = 0; while (x) { n++; x >>= 1; } return n; }

/* xorshift.Next (sort.go): a uint64 state shifted by the triple 13/17/5 (the shifts of
 * Rust's break_patterns, which Go 1.19's port follows; later Go releases are recalled to
 * use the 64-bit triple 13/7/17).  The Go source is not in this container, so the triple is
 * the one assumption of this restatement not pinned by a fixture: only breakPatterns
 * reads it, i.e. only after an unbalanced partition; go_sort_stats counts those calls so
 * a test can state whether a workload depends on it. */
static uint64_t xorshift_next(uint64_t* r) {
    *r ^= *r << 13;
    *r ^= *r >> 17;
    *r ^= *r << 5;
    return *r;
}


/* breakPatterns_func */
static void break_patterns(gs_elem* d, int64_t a, int64_t b) {
    int64_t length = b - a;
    gs_break_calls++;
    if (length >= 8) {
        uint64_t random = (uint64_t)length;
        uint64_t modulus = (uint64_t)1 << bits_len((uint64_t)length);   /* nextPowerOfTwo */
        int64_t idx = a + (length / 4) * 2 - 1;
        for (int i = 0; i < 3; i++) {
            int64_t other = (int64_t)(xorshift_next(&random) & (modulus - 1));
            if (other >= length) other -= length;
            gs_swap(d, idx - 1 + i, a + other);
        }
    }
}

/* order2_func / median_func / medianAdjacent_func */
static void order2(const gs_elem* d, int64_t* a, int64_t* b, int* swaps) {
    if (gs_less(d, *b, *a)) { int64_t t = *a; *a = *b; *b = t; (*swaps)++; }
}
static int64_t median3(const gs_elem* d, int64_t a, int64_t b, int64_t c, int* swaps) {
    order2(d, &a, &b, swaps);
    order2(d, &b, &c, swaps);
    order2(d, &a, &b, swaps);
    return b;
}
static int64_t median_adjacent(const gs_elem* d, int64_t a, int* swaps) { return median3(d, a - 1, a, a + 1, swaps); }

/* choosePivot_func */
static int64_t choose_pivot(const gs_elem* d, int64_t a, int64_t b, int* hint) {
    const int64_t shortestNinther = 50;
    const int maxSwaps = 4 * 3;
    int64_t l = b - a;
    int swaps = 0;
    int64_t i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
        if (l >= shortestNinther) {
            i = median_adjacent(d, i, &swaps);
            j = median_adjacent(d, j, &swaps);
            k = median_adjacent(d, k, &swaps);
        }
        j = median3(d, i, j, k, &swaps);
    }
    *hint = swaps == 0 ? increasingHint : swaps == maxSwaps ? decreasingHint : unknownHint;
    return j;
}

/* reverseRange_func */
static void reverse_range(gs_elem* d, int64_t a, int64_t b) {
    for (int64_t i = a, j = b - 1; i < j; i++, j--) gs_swap(d, i, j);
}

/* partialInsertionSort_func */
static int partial_insertion_sort(gs_elem* d, int64_t a, int64_t b) {
    const int maxSteps = 5;
    const int64_t shortestShifting = 50;
    int64_t i = a + 1;
    for (int s = 0; s < maxSteps; s++) {
        while (i < b && !gs_less(d, i, i - 1)) i++;
        if (i == b) return 1;
        if (b - a < shortestShifting) return 0;
        gs_swap(d, i, i - 1);
        if (i - a >= 2) {                                  /* shift the smaller one left */
            for (int64_t j = i - 1; j >= 1; j--) {
                if (!gs_less(d, j, j - 1)) break;
                gs_swap(d, j, j - 1);
            }
        }
        if (b - i >= 2) {                                  /* shift the greater one right */
            for (int64_t j = i + 1; j < b; j++) {
                if (!gs_less(d, j, j - 1)) break;
                gs_swap(d, j, j - 1);
            }
        }
    }
    return 0;
}

/* partition_func */
static int64_t partition(gs_elem* d, int64_t a, int64_t b, int64_t pivot, int* already) {
    gs_swap(d, a, pivot);
    int64_t i = a + 1, j = b - 1;
    while (i <= j && gs_less(d, i, a)) i++;
    while (i <= j && !gs_less(d, j, a)) j--;
    if (i > j) {
        gs_swap(d, j, a);
        *already = 1;
        return j;
    }
    gs_swap(d, i, j);
    i++;
    j--;
    for (;;) {
        while (i <= j && gs_less(d, i, a)) i++;
        while (i <= j && !gs_less(d, j, a)) j--;
        if (i > j) break;
        gs_swap(d, i, j);
        i++;
        j--;
    }
    gs_swap(d, j, a);
    *already = 0;
    return j;
}

/* partitionEqual_func */
static int64_t partition_equal(gs_elem* d, int64_t a, int64_t b, int64_t pivot) {
    gs_swap(d, a, pivot);
    int64_t i = a + 1, j = b - 1;
    for (;;) {
        while (i <= j && !gs_less(d, a, i)) i++;
        while (i <= j && gs_less(d, a, j)) j--;
        if (i > j) break;
        gs_swap(d, i, j);
        i++;
        j--;
    }
    return i;
}

/* pdqsort_func */
static void pdqsort(gs_elem* d, int64_t a, int64_t b, int limit) {
    const int64_t maxInsertion = 12;
    int wasBalanced = 1, wasPartitioned = 1;
    for (;;) {
        int64_t length = b - a;
        if (length <= maxInsertion) {
            insertion_sort(d, a, b);
            return;
        }
        if (limit == 0) {
            heap_sort(d, a, b);
            return;
        }
        if (!wasBalanced) {
            break_patterns(d, a, b);
            limit--;
        }
        int hint;
        int64_t pivot = choose_pivot(d, a, b, &hint);
        if (hint == decreasingHint) {
            reverse_range(d, a, b);
            pivot = (b - 1) - (pivot - a);
            hint = increasingHint;
        }
        if (wasBalanced && wasPartitioned && hint == increasingHint) {
            if (partial_insertion_sort(d, a, b)) return;
        }
        if (a > 0 && !gs_less(d, a - 1, pivot)) {
            int64_t mid = partition_equal(d, a, b, pivot);
            a = mid;
            continue;
        }
        int already;
        int64_t mid = partition(d, a, b, pivot, &already);
        wasPartitioned = already;
        int64_t leftLen = mid - a, rightLen = b - mid;
        int64_t balanceThreshold = length / 8;
        if (leftLen < rightLen) {
            wasBalanced = leftLen >= balanceThreshold;
            pdqsort(d, a, mid, limit);
            a = mid + 1;
        } else {
            wasBalanced = rightLen >= balanceThreshold;
            pdqsort(d, mid + 1, b, limit);
            b = mid;
        }
    }
}

/* sort.Slice(x, less) with less(i, j) = key[i] > key[j] on elements in their input order;
 * perm[k] = input index of the element sorted to position k.  limit > 0 replaces the
 * initial recursion limit bits.Len(n) (test hook: reaches heapSort). */
void go_sort_slice_desc_limit(const double* key, int32_t n, int32_t limit, int32_t* perm) {
    gs_elem* d = malloc(sizeof(gs_elem) * (size_t)(n > 0 ? n : 1));
    for (int32_t i = 0; i < n; i++) { d[i].key = key[i]; d[i].idx = i; }
    pdqsort(d, 0, n, limit > 0 ? limit : bits_len((uint64_t)n));
    for (int32_t i = 0; i < n; i++) perm[i] = d[i].idx;
    free(d);
}

/* sort.Slice itself: the initial limit is bits.Len(n) */
void go_sort_slice_desc(const double* key, int32_t n, int32_t* perm) { go_sort_slice_desc_limit(key, n, 0, perm); }
