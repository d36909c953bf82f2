// uvector.h -- std::vector whose resize() leaves trivial elements uninitialised.  Large host
// buffers (decompressed BAM streams, record arenas, scan batches) are filled by parallel workers; a
// zero-fill would be a serial first pass over every page.
#pragma once
#include <cstdint>
#include <memory>
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

}  // namespace oge
