// Strict parsing of the MADPOSE_* switches (A/B and diagnostic knobs of the engine).
//
// An unset variable gives the default.  A set one must parse completely and lie in its
// range, otherwise std::invalid_argument names the variable and the value: the C ABI
// turns that into MP_EINVAL and Python into ValueError.  (Before, atoi / atof read a
// typo or a Python repr such as "np.float64(4.0)" silently as 0 / 1.0.)
//
// Presence-only diagnostics (MADPOSE_TRACE, MADPOSE_LO_TIMING, MADPOSE_SWEEP_TIMING) and
// the file / range values (MADPOSE_COUNT_DUMP, MADPOSE_MODEL_DUMP, MADPOSE_TIMELINE) are
// read where they are used.
#pragma once
#include <cerrno>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace mp {

[[noreturn]] inline void env_reject(const char *name, const char *val, const char *want) {
    throw std::invalid_argument(std::string(name) + "=\"" + val + "\": " + want);
}

// integer in [lo, hi]
inline long long env_int(const char *name, long long def, long long lo, long long hi) {
    const char *e = std::getenv(name);
    if (!e) return def;
    char *end = nullptr;
    errno = 0;
    const long long v = std::strtoll(e, &end, 10);
    if (end == e || *end != '\0' || errno == ERANGE) env_reject(name, e, "not an integer");
    if (v < lo || v > hi)
        env_reject(name, e, ("out of range [" + std::to_string(lo) + ", " + std::to_string(hi) + "]").c_str());
    return v;
}

// finite double in [lo, hi]
inline double env_real(const char *name, double def, double lo, double hi) {
    const char *e = std::getenv(name);
    if (!e) return def;
    char *end = nullptr;
    errno = 0;
    const double v = std::strtod(e, &end);
    if (end == e || *end != '\0' || errno == ERANGE || !(v == v)) env_reject(name, e, "not a number");
    if (!(v >= lo && v <= hi)) env_reject(name, e, "out of range");
    return v;
}

// "0" or "1"
inline bool env_flag(const char *name, bool def) {
    const char *e = std::getenv(name);
    if (!e) return def;
    if (e[0] == '0' && e[1] == '\0') return false;
    if (e[0] == '1' && e[1] == '\0') return true;
    env_reject(name, e, "expected 0 or 1");
}

// "avx2" (the 4-wide host path, for A/B) or unset
inline bool env_avx2(const char *name) {
    const char *e = std::getenv(name);
    if (!e) return false;
    if (std::string(e) == "avx2") return true;
    env_reject(name, e, "expected avx2");
}

} // namespace mp
