// uvector.h -- std::vector whose resize() leaves trivial elements uninitialised.  Large host
// buffers (decompressed BAM streams, record arenas, scan batches) are filled by parallel workers; a
// zero-fill would be a serial first pass over every page.  hvector: the same on 2 MiB pages.
#pragma once
#include <sys/mman.h>

#include <cstdint>
#include <cstdlib>
#include <memory>
#include <new>
#include <utility>
#include <vector>

namespace oge {

template <class T>
struct UninitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        typedef UninitAlloc<U> other;
    };
    UninitAlloc() = default;
    template <class U>
    UninitAlloc(const UninitAlloc<U> &) {}
    template <class U>
    void construct(U *p) noexcept {
        ::new ((void *)p) U;
    }
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        ::new ((void *)p) U(std::forward<A>(a)...);
    }
};
template <class T>
using uvector = std::vector<T, UninitAlloc<T>>;
typedef uvector<uint8_t> bytevec;

// 2 MiB pages for [p, p + bytes) where the kernel allows them (one fault per 2 MiB instead of 512)
inline void advise_huge(void *p, size_t bytes) {
    const uintptr_t a = ((uintptr_t)p + (2ull << 20) - 1) & ~(uintptr_t)((2ull << 20) - 1);
    const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)((2ull << 20) - 1);
    if (e > a) madvise((void *)a, e - a, MADV_HUGEPAGE);
}
// malloc, with buffers of 4 MiB and up 2 MiB-aligned on 2 MiB pages; release with free()
inline void *big_alloc(size_t bytes) {
    void *p = nullptr;
    if (bytes >= (4ull << 20)) {
        if (posix_memalign(&p, 2ull << 20, bytes)) return nullptr;
        advise_huge(p, bytes);
        return p;
    }
    return std::malloc(bytes ? bytes : 1);
}
// uvector on big_alloc: per-read arrays that a process's first call touches for the first time (realign.cpp)
template <class T>
struct HugeAlloc : UninitAlloc<T> {
    using value_type = T;
    template <class U>
    struct rebind {
        typedef HugeAlloc<U> other;
    };
    HugeAlloc() = default;
    template <class U>
    HugeAlloc(const HugeAlloc<U> &) {}
    T *allocate(size_t n) {
        T *p = (T *)big_alloc(n * sizeof(T));
        if (!p) throw std::bad_alloc();
        return p;
    }
    void deallocate(T *p, size_t) { std::free(p); }
};
template <class T, class U>
bool operator==(const HugeAlloc<T> &, const HugeAlloc<U> &) { return true; }
template <class T, class U>
bool operator!=(const HugeAlloc<T> &, const HugeAlloc<U> &) { return false; }
template <class T>
using hvector = std::vector<T, HugeAlloc<T>>;

}  // namespace oge
