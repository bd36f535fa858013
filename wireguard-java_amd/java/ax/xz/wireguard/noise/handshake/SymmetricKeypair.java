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
 * The keys live in the MI355X key table (wg_keys_set); the per-packet calls are
 * synchronous device round trips. {@link #sendBatch()} / {@link #receiveBatch()}
 * expose the additive batch API a batching TransportManager uses (INTEGRATION.md).
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
	private volatile long sendCounter = 0;
	private volatile boolean cleaned = false;

	SymmetricKeypair(byte[] sendKeyBytes, byte[] receiveKeyBytes) {
		int slots = TransportBatch.installKeys(MemorySegment.ofArray(sendKeyBytes), MemorySegment.ofArray(receiveKeyBytes));
		this.sendSlot = slots >>> 16;
		this.receiveSlot = slots & 0xffff;
		int s = sendSlot, r = receiveSlot;
		cleaner.register(this, () -> TransportBatch.releaseKeys(s, r));
	}

	public long cipher(MemorySegment src, MemorySegment dst) {
		var counter = (long) SEND_COUNTER.getAndAdd(this, 1);
		TransportBatch.seal1(sendSlot, counter, src, dst.asSlice(0, src.byteSize() + 16));
		return counter;
	}

	public void decipher(long counter, MemorySegment src, MemorySegment dst) throws BadPaddingException {
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
		if (!cleaned) {
			cleaned = true;
			TransportBatch.releaseKeys(sendSlot, receiveSlot);
		}
	}
}
