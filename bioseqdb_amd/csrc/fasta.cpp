// fasta.cpp -- the FASTA reader of the bulk loader (reference:
// bioseqdb-import/main.cpp:48-71).  Lines are std::getline lines (split at '\n' only, so a '\r' stays in
// the line; no empty line after a final '\n').  A line starting with '>' submits the current record and
// names the next one (the rest of the line); any other line is upper-cased (std::toupper, C locale) and
// appended to the current sequence.  A record whose sequence is empty is not emitted, and its name is
// dropped (try_submit_sequence, :52-60).  The database INSERT is the caller's.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/bsq.h"

extern "C" int bsq_fasta_parse(const char *data, int64_t size, char **seq, int64_t **seq_off, char **names,
                               int64_t **name_off, int64_t *n_records)
{
    if ((size && !data) || size < 0 || !seq || !seq_off || !names || !name_off || !n_records) return BSQ_E_INVALID;
    std::string s, nm, cur_name;
    std::vector<int64_t> so{0}, no{0};
    s.reserve((size_t)size);
    size_t rec_start = 0;
    auto submit = [&] {
        if (s.size() > rec_start) {
            nm += cur_name;
            so.push_back((int64_t)s.size());
            no.push_back((int64_t)nm.size());
            rec_start = s.size();
        }
        cur_name.clear();
    };
    const char *p = data, *end = data + size;
    while (p < end) {
        const char *q = static_cast<const char *>(memchr(p, '\n', (size_t)(end - p)));
        const char *le = q ? q : end;
        if (le > p && *p == '>') {
            submit();
            cur_name.assign(p + 1, le);
        } else {
            const size_t at = s.size();
            s.append(p, le);
            for (size_t i = at; i < s.size(); ++i)
                if (s[i] >= 'a' && s[i] <= 'z') s[i] = (char)(s[i] - 'a' + 'A');
        }
        p = q ? q + 1 : end;
    }
    submit();
    *n_records = (int64_t)so.size() - 1;
    *seq = static_cast<char *>(malloc(s.size() + 1));
    *names = static_cast<char *>(malloc(nm.size() + 1));
    *seq_off = static_cast<int64_t *>(malloc(so.size() * 8));
    *name_off = static_cast<int64_t *>(malloc(no.size() * 8));
    if (!*seq || !*names || !*seq_off || !*name_off) {
        free(*seq); free(*names); free(*seq_off); free(*name_off);
        *seq = *names = nullptr; *seq_off = *name_off = nullptr;
        return BSQ_E_NOMEM;
    }
    memcpy(*seq, s.data(), s.size()); (*seq)[s.size()] = 0;
    memcpy(*names, nm.data(), nm.size()); (*names)[nm.size()] = 0;
    memcpy(*seq_off, so.data(), so.size() * 8);
    memcpy(*name_off, no.data(), no.size() * 8);
    return BSQ_OK;
}
