// Shared host-side helpers of the C ABI translation units (engine.cpp, vocos.cpp).
#pragma once
#include <string>

// Sets the thread-local message returned by f5h_last_error() and returns `code`.
int f5h_internal_fail(int code, const std::string& msg);
