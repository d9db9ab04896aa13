// work_pool.hpp — the host driver's fork-join pool for its parallel loops over reads.
//
// The reference parallelises its per-read phases with OpenMP (bt2_search.cpp:2429-2814).
// Here the loops run between GPU launches, with the scheduler thread doing serial work
// (launch calls, retiring, output) in between; workers therefore sleep on a condition
// variable instead of spinning (an OpenMP team's default spin-wait takes CPU from the
// HIP runtime and the SAM writer, and its policy can only be set from the environment).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

namespace bt2x {
namespace host {

class WorkPool {
public:
	explicit WorkPool(int nthreads) {
		const int nw = std::max(1, nthreads) - 1;
		for(int i = 0; i < nw; i++) th_.emplace_back([this] { worker(); });
	}
	~WorkPool() {
		{ std::lock_guard<std::mutex> g(mu_); stop_ = true; }
		cv_.notify_all();
		for(std::thread& t : th_) t.join();
	}
	WorkPool(const WorkPool&) = delete;
	WorkPool& operator=(const WorkPool&) = delete;
	int threads() const { return (int)th_.size() + 1; }

	// f(i) for i in [0, n), chunks of `chunk` indices handed out dynamically; the calling
	// thread takes part.  The first exception thrown by f is rethrown here.
	template<class F> void parallel_for(long n, long chunk, F&& f) {
		if(n <= 0) return;
		using Fn = std::remove_reference_t<F>;
		if(th_.empty() || n <= chunk) { for(long i = 0; i < n; i++) f(i); return; }
		auto thunk = [](void* c, long b, long e) { Fn& ff = *static_cast<Fn*>(c); for(long i = b; i < e; i++) ff(i); };
		run(n, std::max(1L, chunk), thunk, (void*)&f);
	}

private:
	using Thunk = void (*)(void*, long, long);
	void run(long n, long chunk, Thunk fn, void* ctx) {
		{
			std::lock_guard<std::mutex> g(mu_);
			fn_ = fn; ctx_ = ctx; n_ = n; chunk_ = chunk;
			next_.store(0, std::memory_order_relaxed);
			pending_ = (int)th_.size();            // every worker checks in once per job
			err_ = nullptr;
			gen_++;
		}
		cv_.notify_all();
		chunks();
		std::unique_lock<std::mutex> g(mu_);
		done_.wait(g, [&] { return pending_ == 0; });
		if(err_) std::rethrow_exception(err_);
	}
	void chunks() {
		try {
			for(;;) {
				const long b = next_.fetch_add(chunk_, std::memory_order_relaxed);
				if(b >= n_) break;
				fn_(ctx_, b, std::min(n_, b + chunk_));
			}
		} catch(...) {
			std::lock_guard<std::mutex> g(mu_);
			if(!err_) err_ = std::current_exception();
			next_.store(n_, std::memory_order_relaxed);   // stop handing out work
		}
	}
	void worker() {
		uint64_t seen = 0;
		for(;;) {
			{
				std::unique_lock<std::mutex> g(mu_);
				cv_.wait(g, [&] { return stop_ || gen_ != seen; });
				if(stop_) return;
				seen = gen_;
			}
			chunks();
			std::lock_guard<std::mutex> g(mu_);
			if(--pending_ == 0) done_.notify_one();
		}
	}
	std::vector<std::thread> th_;
	std::mutex mu_;
	std::condition_variable cv_, done_;
	uint64_t gen_ = 0;
	bool stop_ = false;
	int pending_ = 0;
	Thunk fn_ = nullptr;
	void* ctx_ = nullptr;
	long n_ = 0, chunk_ = 1;
	std::atomic<long> next_{0};
	std::exception_ptr err_;
};

} // namespace host
} // namespace bt2x
