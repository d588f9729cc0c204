// Internal helpers shared by the host and device translation units.
#pragma once
#include <string>

namespace flexar {
void set_error(const std::string& msg);
}
