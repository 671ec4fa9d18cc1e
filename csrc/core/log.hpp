// Leveled logging with the reference's line format
// "[HH:MM:SS][pid][LEVEL] msg" (reference erp_utilities.cpp:82-145):
// debug -> stdout, everything else -> stderr, showLevel=false prints "------> ".
#pragma once

#include <cstdarg>

namespace brp {

enum LogLevel : int { LOG_ERROR = 1, LOG_WARN = 2, LOG_INFO = 3, LOG_DEBUG = 4 };

// Runtime threshold (reference uses a compile-time LOGLEVEL). Defaults to
// LOG_INFO; BRP_LOGLEVEL=1..4 or set_log_level() override it.
void set_log_level(int level);
int log_level();

void log_message(LogLevel level, bool show_level, const char* fmt, ...)
    __attribute__((format(printf, 3, 4)));
void log_vmessage(LogLevel level, bool show_level, const char* fmt, va_list ap);

}  // namespace brp
