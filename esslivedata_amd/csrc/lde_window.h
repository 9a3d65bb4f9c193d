// lde_window.h -- host choice of the SIEVE hot rows' TOA window (no HIP).
//
// A hot row holds the bins [lo, lo + w) of its screen, so narrower rows fit
// more screens into the same LDS.  From a sample (events per screen, events
// per TOA bin) the choice maximizes the estimated hot fraction
//   (share of the top-H screens) x (share of the window's bins)
// over w (and the best lo for each w), against whole rows (w = T); only a gain
// of at least `min_gain` of the events changes the rows.  Counting stays
// exact whatever the choice: a hot screen's event outside the window leaves
// as a cold key.
#ifndef LDE_WINDOW_H
#define LDE_WINDOW_H

#include <stdint.h>

#include <algorithm>
#include <functional>
#include <vector>

namespace lde {

struct HotWindow {
    int rows, w, lo;
    double win;   // sampled share of the times inside [lo, lo + w)
    double est;   // estimated hot fraction of the events
};

// rows_for(w, lo): the most rows of w bins starting at lo that fit the LDS
inline HotWindow choose_hot_window(const uint32_t *screen_cnt, long long S, const uint32_t *toa_hist,
                                   int T, int whole_rows,
                                   const std::function<int(int, int)> &rows_for,
                                   double min_gain = 0.005) {
    std::vector<uint32_t> c(screen_cnt, screen_cnt + S);
    std::sort(c.begin(), c.end(), std::greater<uint32_t>());
    std::vector<double> top((size_t)S + 1, 0.0);
    for (long long i = 0; i < S; ++i) top[(size_t)i + 1] = top[(size_t)i] + c[(size_t)i];
    std::vector<double> tp((size_t)T + 1, 0.0);
    for (int b = 0; b < T; ++b) tp[(size_t)b + 1] = tp[(size_t)b] + toa_hist[b];
    auto share = [&](long long H) {
        return top[(size_t)S] > 0 ? top[(size_t)std::min(H, S)] / top[(size_t)S] : 0.0;
    };
    HotWindow best{whole_rows, T, 0, 1.0, share(whole_rows)};
    if (top[(size_t)S] <= 0 || tp[(size_t)T] <= 0) return best;
    for (int w = T - 1; w >= std::max(8, T / 4); --w) {
        int lo = 0;
        for (int l = 1; l + w <= T; ++l)
            if (tp[(size_t)l + w] - tp[(size_t)l] > tp[(size_t)lo + w] - tp[(size_t)lo]) lo = l;
        const int H = rows_for(w, lo);
        if (H < 8) continue;
        const double win = (tp[(size_t)lo + w] - tp[(size_t)lo]) / tp[(size_t)T];
        const double est = share(H) * win;
        if (est > best.est + min_gain) best = HotWindow{H, w, lo, win, est};
    }
    return best;
}

}  // namespace lde

#endif  // LDE_WINDOW_H
