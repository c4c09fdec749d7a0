// Test scaffold: the slice of libe's <e/slice.h> that hyperdex_amd/hash.h uses
// (data(), size()).  The real daemon build uses libe itself.
#ifndef e_slice_h_
#define e_slice_h_
#include <stddef.h>
#include <stdint.h>
#include <string.h>
namespace e {
class slice {
  public:
    slice() : m_data(NULL), m_sz(0) {}
    slice(const uint8_t* d, size_t sz) : m_data(d), m_sz(sz) {}
    slice(const char* s) : m_data(reinterpret_cast<const uint8_t*>(s)), m_sz(strlen(s)) {}
    const uint8_t* data() const { return m_data; }
    size_t size() const { return m_sz; }
    bool empty() const { return m_sz == 0; }
  private:
    const uint8_t* m_data;
    size_t m_sz;
};
}  // namespace e
#endif
