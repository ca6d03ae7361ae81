// Library-wide entry points: error text, version, build limits.
#include "sra_common.hpp"

namespace sra {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

const char* last_error() { return g_err; }

}  // namespace sra

extern "C" const char* sra_last_error(void) { return sra::last_error(); }
extern "C" int sra_version(void) { return 100; }
extern "C" int sra_max_register_clients(void) { return 128; }

extern "C" int sra_row_fault_count(int32_t reset, uint32_t* count) {
  SRA_REQUIRE(count != nullptr, SRA_ERR_ARG, "null count pointer");
  *count = sra::krum_row_faults(reset != 0) + sra::bulyan_row_faults(reset != 0);
  return SRA_OK;
}
