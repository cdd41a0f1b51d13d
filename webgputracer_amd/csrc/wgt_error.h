// wgt_error.h — thread-local error message behind wgt_last_error(NULL).
#pragma once
#include <string>
namespace wgt {
void set_thread_error(const std::string& msg);
}
