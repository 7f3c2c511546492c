// libbert's message sink.  Every error line the library prints goes to stderr,
// as the reference prints its errors (bert.cpp:847-853, fprintf(stderr, ...)),
// and -- when BERT_LOG=<file> is set -- is also appended to that file with one
// unbuffered write(2) per line, so the cause of a failure survives a process
// that dies right after it (pytest's fd capture loses stderr on an abort).
// Stage lines of the load path go to the file only (emb::trace); informational
// lines (emb::infof) to stdout only.
#include "host_common.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <mutex>

namespace emb {
namespace {

// BERT_LOG=<path>: append to that file.  BERT_LOG=fd:<n>:<dev>:<ino>: write to the
// inherited descriptor n when it still is that file (the test runner hands over a
// duplicate of its own stderr, so library lines share its file offset and land
// in order in its log; a child process where n is absent or reused ignores it).
int log_fd()
{
    static const int fd = [] {
        const char *p = std::getenv("BERT_LOG");
        if (!p || !*p) return -1;
        if (std::strncmp(p, "fd:", 3) == 0) {
            int n = -1;
            unsigned long long dev = 0, ino = 0;
            if (std::sscanf(p + 3, "%d:%llu:%llu", &n, &dev, &ino) != 3 || n < 0) return -1;
            struct stat st;
            if (::fstat(n, &st) != 0 || (unsigned long long)st.st_dev != dev || (unsigned long long)st.st_ino != ino)
                return -1;
            return n;
        }
        return ::open(p, O_WRONLY | O_APPEND | O_CREAT | O_CLOEXEC, 0644);
    }();
    return fd;
}

void emit(FILE *stream, const char *fmt, va_list ap)
{
    char buf[1024];
    int n = std::vsnprintf(buf, sizeof buf, fmt, ap);
    if (n < 0) return;
    if ((size_t)n >= sizeof buf) n = (int)sizeof buf - 1;
    if (stream) {
        std::fwrite(buf, 1, (size_t)n, stream);
        std::fflush(stream);
    }
    const int fd = log_fd();
    if (fd >= 0) {
        // one write per line (O_APPEND: lines of concurrent threads never interleave)
        char line[1100];
        const int m = std::snprintf(line, sizeof line, "[%d] %.*s", (int)::getpid(), n, buf);
        if (m > 0) (void)!::write(fd, line, (size_t)std::min<int>(m, (int)sizeof line - 1));
    }
}

}  // namespace

void errorf(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    emit(stderr, fmt, ap);
    va_end(ap);
}

void infof(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    std::vfprintf(stdout, fmt, ap);   // progress for the caller's stdout only (not BERT_LOG)
    va_end(ap);
    std::fflush(stdout);
}

void trace(const char *fmt, ...)
{
    if (log_fd() < 0) return;
    va_list ap;
    va_start(ap, fmt);
    emit(nullptr, fmt, ap);
    va_end(ap);
}

bool fault_inject(const char *stage)
{
    // BERT_FAULT_INJECT=<stage>[,<stage>...] (tests only): the named load stage
    // throws, so the tests can check that every failure of the load path becomes
    // a NULL context and a message, never an abort
    const char *env = std::getenv("BERT_FAULT_INJECT");   // read per call: a test may clear it
    if (!env || !*env) return false;
    const size_t n = std::strlen(stage);
    for (const char *p = env; *p;) {
        const char *q = std::strchr(p, ',');
        const size_t len = q ? (size_t)(q - p) : std::strlen(p);
        if (len == n && std::strncmp(p, stage, n) == 0) return true;
        if (!q) break;
        p = q + 1;
    }
    return false;
}

}  // namespace emb
