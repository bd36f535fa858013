package ax.xz.wireguard.noise.handshake;

import ax.xz.wireguard.noise.crypto.TransportBatch;

import javax.crypto.AEADBadTagException;
import javax.crypto.BadPaddingException;
import java.lang.foreign.MemorySegment;
import java.lang.invoke.MethodHandles;
import java.lang.invoke.VarHandle;
import java.lang.ref.Cleaner;

/**
 * Drop-in for ax.xz.wireguard.noise.handshake.SymmetricKeypair (reference
 * SymmetricKeypair.java:20-94). Same API and semantics:
 * <ul>
 *   <li>send counters start at 0 and are claimed with an atomic getAndAdd (:37, :64);</li>
 *   <li>nonce = LE64(counter) || 00 00 00 00 — built on the device (:52-61);</li>
 *   <li>cipher(src, dst): dst = ciphertext || tag, returns the counter (:63-74);</li>
 *   <li>decipher(counter, src = ct || tag, dst): AEADBadTagException on a bad tag, dst untouched (:76-83);</li>
 *   <li>clean(): zeroes both keys (:85-93) — here the device key-table slots.</li>
 * </ul>
 * The keys live in the MI355X key table (wg_keys_set). The per-packet calls are
 * synchronous for the caller but batched underneath (wg_seal1 / wg_open1 share
 * device launches with every concurrent caller; INTEGRATION.md §3).
 * {@link #claimCounters(int)}, {@link #sendSlot()} and {@link #receiveSlot()} expose
 * what a batching TransportManager needs for the additive batch API.
 *
 * <p>The key slots are released exactly once: {@link #clean()} runs the Cleaner
 * action itself (Cleanable.clean runs it at most once), so a later garbage collection
 * cannot release slots that a newer keypair already holds.
 */
public final class SymmetricKeypair {
	private static final VarHandle SEND_COUNTER;

	static {
		try {
			SEND_COUNTER = MethodHandles.lookup().findVarHandle(SymmetricKeypair.class, "sendCounter", long.class);
		} catch (NoSuchFieldException | IllegalAccessException e) {
			throw new AssertionError(e);
		}
	}

	private static final Cleaner cleaner = Cleaner.create();

	private final int sendSlot, receiveSlot;
	private final Cleaner.Cleanable cleanable;
	private volatile long sendCounter = 0;
	private volatile boolean cleaned = false;

	SymmetricKeypair(byte[] sendKeyBytes, byte[] receiveKeyBytes) {
		int slots = TransportBatch.installKeys(MemorySegment.ofArray(sendKeyBytes), MemorySegment.ofArray(receiveKeyBytes));
		this.sendSlot = slots >>> 16;
		this.receiveSlot = slots & 0xffff;
		int s = sendSlot, r = receiveSlot;
		// the action must not capture `this`; Cleanable.clean() runs it at most once
		this.cleanable = cleaner.register(this, () -> TransportBatch.releaseKeys(s, r));
	}

	private void checkLive() {
		if (cleaned)  // the reference's keys live in a closed Arena after clean() (:85-93)
			throw new IllegalStateException("SymmetricKeypair used after clean()");
	}

	public long cipher(MemorySegment src, MemorySegment dst) {
		checkLive();
		var counter = (long) SEND_COUNTER.getAndAdd(this, 1);
		TransportBatch.seal1(sendSlot, counter, src, dst.asSlice(0, src.byteSize() + 16));
		return counter;
	}

	public void decipher(long counter, MemorySegment src, MemorySegment dst) throws BadPaddingException {
		checkLive();
		long textLength = src.byteSize() - 16;
		src.asSlice(textLength, 16);  // IndexOutOfBoundsException for a short src, like the reference
		if (!TransportBatch.open1(receiveSlot, counter, src, dst.asSlice(0, textLength)))
			throw new AEADBadTagException("Invalid tag");
	}

	/** Claims {@code n} consecutive send counters for a batch (same atomic as cipher). */
	public long claimCounters(int n) {
		return (long) SEND_COUNTER.getAndAdd(this, (long) n);
	}

	public int sendSlot() {
		return sendSlot;
	}

	public int receiveSlot() {
		return receiveSlot;
	}

	public void clean() {
		cleaned = true;
		cleanable.clean();  // zeroes and releases both slots, once
	}
}
