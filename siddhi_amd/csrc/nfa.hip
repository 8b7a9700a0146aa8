// nfa.hip — execution path SG_PATH_NFA (general per-partition NFA interpreter). [in progress]
#include "runtime.hpp"
namespace sg {
std::unique_ptr<Exec> make_nfa(App&, int, const J&, std::string& why) { why = "not built yet"; return nullptr; }
}
