// window_agg.hip — execution path SG_PATH_WINDOW_AGG. [in progress]
#include "runtime.hpp"
namespace sg {
std::unique_ptr<Exec> make_window_agg(App&, int, const J&, std::string& why) { why = "not built yet"; return nullptr; }
}
