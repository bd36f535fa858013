package ax.xz.wireguard.noise.crypto;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;

import static java.lang.foreign.ValueLayout.*;

/**
 * Asynchronous batch submission (wg_queue, include/wgaead.h): the batching TransportManager of
 * INTEGRATION.md §3. The reference hands every packet to a ForkJoinPool worker that calls
 * cipher / decipher and then enqueues the result for the UDP / tun worker
 * (TransportManager.java:41,70-93,137-158; EstablishedSession.java:88-90). With a queue the worker
 * only submits (a copy into a pinned ring, no wait for the crypto) and the UDP / tun worker reaps the
 * finished packets; one native thread per queue batches them into kernel launches.
 *
 * <pre>
 * // outgoing: FJP workers
 * long ctr = keypair.claimCounters(1);                    // SymmetricKeypair's getAndAdd (:64)
 * sealQ.submit(keypair.sendSlot(), ctr, plaintext, tag);
 * // UDP worker: reap, write the 16-B header (TransportPacket.java:30-35), send, give the slots back
 * int n = sealQ.reap(256, 1000);
 * for (int i = 0; i < n; i++) send(sealQ.user(i), sealQ.counter(i), sealQ.data(i));   // ct || tag
 * sealQ.done(n);
 * </pre>
 *
 * Not compiled here: the build image and the GPU box have no JDK (DESIGN.md §1). The downcall
 * descriptors are checked against the C header by tests/test_java_binding.py.
 */
public final class TransportQueue implements AutoCloseable {
	/** wg_completion: {user u64, counter u64, data ptr, len u32, status u32, key_slot u32, slot u32, submit_ns u64}. */
	static final long COMPLETION_SIZE = 48;
	/** wg_submit: {user u64, counter u64, data ptr, len u32, key_slot u32}. */
	static final long SUBMIT_SIZE = 32;

	private final MemorySegment q;
	private final boolean open;
	private final Arena arena = Arena.ofShared();
	private final MemorySegment comps;
	private final int cap;

	/**
	 * @param open     false: a seal queue (plaintext in, ct || tag out); true: an open queue
	 * @param capacity ring slots (0 = 65536)
	 * @param maxLen   largest payload (0 = 2032, the reference's incoming limit)
	 * @param reapMax  completions one reap() returns at most
	 */
	public TransportQueue(boolean open, int capacity, int maxLen, int reapMax) {
		this.open = open;
		this.cap = reapMax;
		try (var a = Arena.ofConfined()) {
			var out = a.allocate(ADDRESS);
			WgAead.check((int) WgAead.QUEUE_CREATE.invokeExact(WgAead.CTX, open ? WgAead.WG_MODE_OPEN : WgAead.WG_MODE_SEAL,
				capacity, maxLen, 0, out));
			q = out.get(ADDRESS, 0);
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
		comps = arena.allocate(COMPLETION_SIZE * reapMax, 16);
	}

	/** Queue one packet: plaintext for a seal queue, ct || tag (len + 16 bytes) for an open queue. */
	public void submit(int keySlot, long counter, MemorySegment src, long user) {
		final int len = (int) src.byteSize() - (open ? 16 : 0);
		try {
			WgAead.check(open ? (int) WgAead.SUBMIT_OPEN.invokeExact(q, keySlot, counter, src, len, user)
			                  : (int) WgAead.SUBMIT_SEAL.invokeExact(q, keySlot, counter, src, len, user));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/**
	 * Queue n packets in one call (wg_submit_seal_n / wg_submit_open_n: one lane lock and one publication
	 * per run of free slots instead of per packet), e.g. everything one receive burst or one reap() of the
	 * peer's queue returned. Returns how many were queued: n, or fewer when the submit timeout ran out.
	 */
	public int submitAll(int[] keySlots, long[] counters, MemorySegment[] srcs, long[] users, int n) {
		try (var a = Arena.ofConfined()) {
			var sub = a.allocate(SUBMIT_SIZE * Math.max(n, 1), 16);
			for (int i = 0; i < n; i++) {
				final long o = i * SUBMIT_SIZE;
				sub.set(JAVA_LONG, o, users[i]);
				sub.set(JAVA_LONG, o + 8, counters[i]);
				sub.set(ADDRESS, o + 16, srcs[i]);
				sub.set(JAVA_INT, o + 24, (int) srcs[i].byteSize() - (open ? 16 : 0));
				sub.set(JAVA_INT, o + 28, keySlots[i]);
			}
			return WgAead.check(open ? (int) WgAead.SUBMIT_OPEN_N.invokeExact(q, sub, n)
			                         : (int) WgAead.SUBMIT_SEAL_N.invokeExact(q, sub, n));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/**
	 * How long submit() waits for a free ring slot before it fails (wg_queue_set_submit_timeout; WG_EAGAIN,
	 * thrown as a RuntimeException by WgAead.check): a stalled UDP / tun worker then cannot block every
	 * ForkJoinPool worker for good. 0 (the default): wait without bound.
	 */
	public void submitTimeout(int timeoutUs) {
		try {
			WgAead.check((int) WgAead.QUEUE_SUBMIT_TIMEOUT.invokeExact(q, timeoutUs));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	/** Up to reapMax finished packets (waits up to timeoutUs for the first); read them with user/data/status. */
	public int reap(int max, int timeoutUs) {
		try {
			return WgAead.check((int) WgAead.REAP.invokeExact(q, comps, Math.min(max, cap), timeoutUs));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	public long user(int i) { return comps.get(JAVA_LONG, i * COMPLETION_SIZE); }

	public long counter(int i) { return comps.get(JAVA_LONG, i * COMPLETION_SIZE + 8); }

	/** WG_PKT_OK, WG_PKT_BADTAG (open: the reference's drop-and-log path, TransportManager.java:89) or 255. */
	public int status(int i) { return comps.get(JAVA_INT, i * COMPLETION_SIZE + 28); }

	/** The result in the pinned ring: ct || tag (seal) or the plaintext (open); valid until done(). */
	public MemorySegment data(int i) {
		final int len = comps.get(JAVA_INT, i * COMPLETION_SIZE + 24);
		return comps.get(ADDRESS, i * COMPLETION_SIZE + 16).reinterpret(len + (open ? 0 : 16));
	}

	/** The first n completions of the last reap() are sent / written: their ring slots are reused. */
	public void done(int n) {
		try {
			WgAead.check((int) WgAead.REAP_DONE.invokeExact(q, comps, n));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
	}

	@Override
	public void close() {
		try {
			WgAead.check((int) WgAead.QUEUE_DESTROY.invokeExact(q));
		} catch (RuntimeException e) {
			throw e;
		} catch (Throwable e) {
			throw new RuntimeException(e);
		}
		arena.close();
	}
}
