"""Text front end of the synthesizer: symbols, cleaners, text -> id sequence.

Restates the reference's ``synthesizer/utils/symbols.py`` (symbol table :8-17),
``synthesizer/utils/text.py`` (``text_to_sequence`` :26-53, ``sequence_to_text`` :56-66) and
``synthesizer/utils/cleaners.py`` (abbreviations :22-51, ``english_cleaners`` :90-97).

Two third-party steps of the reference are absent from this image and are restated here:
``unidecode`` (transliteration; here Unicode NFKD decomposition with non-ASCII dropped, which
agrees with unidecode on accented Latin text) and ``inflect`` (number words; here
``number_to_words`` below, following inflect's documented output: hyphenated tens, comma
between thousands groups, optional "and", ``group=2`` year reading with ``zero="oh"``). Text
without digits or non-ASCII characters is pinned against the reference's own code
(tests/golden/e2e_text.json); numbers and transliteration are "parity unpinned".
"""
import re
import unicodedata

_pad = "_"
_punctuation = "!'\"(),-.:;? "
_eos = "~"
_characters = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
symbols = [_pad, _eos] + list(_characters) + list(_punctuation)
_symbol_to_id = {s: i for i, s in enumerate(symbols)}
_id_to_symbol = {i: s for i, s in enumerate(symbols)}

_whitespace_re = re.compile(r"\s+")
_curly_re = re.compile(r"(.*?)\{(.+?)\}(.*)")
_abbreviations = [(re.compile("\\b%s\\." % a, re.IGNORECASE), b) for a, b in [
    ("mrs", "misess"), ("mr", "mister"), ("dr", "doctor"), ("st", "saint"), ("co", "company"),
    ("jr", "junior"), ("maj", "major"), ("gen", "general"), ("drs", "doctors"),
    ("rev", "reverend"), ("lt", "lieutenant"), ("hon", "honorable"), ("sgt", "sergeant"),
    ("capt", "captain"), ("esq", "esquire"), ("ltd", "limited"), ("col", "colonel"),
    ("ft", "fort"), ("mk", "mark"), ("jan", "january"), ("feb", "february"), ("mar", "march"),
    ("apr", "april"), ("aug", "august"), ("sept", "september"), ("oct", "october"),
    ("nov", "november"), ("dec", "december")]]

# --- number words (inflect restatement) --------------------------------------------------
_ONES = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine", "ten",
         "eleven", "twelve", "thirteen", "fourteen", "fifteen", "sixteen", "seventeen",
         "eighteen", "nineteen"]
_TENS = ["", "", "twenty", "thirty", "forty", "fifty", "sixty", "seventy", "eighty", "ninety"]
_GROUPS = ["", " thousand", " million", " billion", " trillion", " quadrillion"]
_ORD = {"one": "first", "two": "second", "three": "third", "five": "fifth", "eight": "eighth",
        "nine": "ninth", "twelve": "twelfth"}


def _below_100(n):
    if n < 20:
        return _ONES[n]
    return _TENS[n // 10] + ("-" + _ONES[n % 10] if n % 10 else "")


def _below_1000(n, andword):
    if n < 100:
        return _below_100(n)
    s = _ONES[n // 100] + " hundred"
    if n % 100:
        s += (" " + andword if andword else "") + " " + _below_100(n % 100)
    return s


def number_to_words(num, andword="and", zero="zero", group=0):
    """Cardinal words of a non-negative integer (inflect.engine().number_to_words subset)."""
    num = int(num)
    if group == 2:  # read in pairs of digits: 1984 -> "nineteen, eighty-four", 1905 -> "..., oh five"
        digits = str(num)
        pairs = [digits[max(0, i - 2):i] for i in range(len(digits), 0, -2)][::-1]
        words = []
        for p in pairs:
            v = int(p)
            words.append(zero + " " + _ONES[v] if len(p) == 2 and p[0] == "0" else _below_100(v))
        return ", ".join(words)
    if num == 0:
        return zero
    groups = []
    g = 0
    while num:
        num, rem = divmod(num, 1000)
        if rem:
            groups.append(_below_1000(rem, andword) + _GROUPS[g])
        g += 1
    return ", ".join(reversed(groups))


def ordinal_words(num):
    w = number_to_words(num)
    head, _, last = w.rpartition(" ")
    sep = " " if head else ""
    if "-" in last:
        a, b = last.rsplit("-", 1)
        last = a + "-" + _ORD.get(b, (b[:-1] + "ieth") if b.endswith("y") else b + "th")
    elif last in _ORD:
        last = _ORD[last]
    elif last.endswith("y"):
        last = last[:-1] + "ieth"
    else:
        last = last + "th"
    return head + sep + last


_comma_number_re = re.compile(r"([0-9][0-9\,]+[0-9])")
_decimal_number_re = re.compile(r"([0-9]+\.[0-9]+)")
_pounds_re = re.compile(r"£([0-9\,]*[0-9]+)")
_dollars_re = re.compile(r"\$([0-9\.\,]*[0-9]+)")
_ordinal_re = re.compile(r"[0-9]+(st|nd|rd|th)")
_number_re = re.compile(r"[0-9]+")


def _dollars(m):
    parts = m.group(1).split(".")
    if len(parts) > 2:
        return m.group(1) + " dollars"
    d = int(parts[0]) if parts[0] else 0
    c = int(parts[1]) if len(parts) > 1 and parts[1] else 0
    du, cu = ("dollar" if d == 1 else "dollars"), ("cent" if c == 1 else "cents")
    if d and c:
        return "%s %s, %s %s" % (d, du, c, cu)
    if d:
        return "%s %s" % (d, du)
    if c:
        return "%s %s" % (c, cu)
    return "zero dollars"


def _number(m):
    n = int(m.group(0))
    if 1000 < n < 3000:
        if n == 2000:
            return "two thousand"
        if 2000 < n < 2010:
            return "two thousand " + number_to_words(n % 100)
        if n % 100 == 0:
            return number_to_words(n // 100) + " hundred"
        return number_to_words(n, andword="", zero="oh", group=2).replace(", ", " ")
    return number_to_words(n, andword="")


def normalize_numbers(text):
    """synthesizer/utils/numbers.py:61-68 (same regex passes, same order)."""
    text = re.sub(_comma_number_re, lambda m: m.group(1).replace(",", ""), text)
    text = re.sub(_pounds_re, r"\1 pounds", text)
    text = re.sub(_dollars_re, _dollars, text)
    text = re.sub(_decimal_number_re, lambda m: m.group(1).replace(".", " point "), text)
    text = re.sub(_ordinal_re, lambda m: ordinal_words(int(m.group(0)[:-2])), text)
    return re.sub(_number_re, _number, text)


# --- cleaners -----------------------------------------------------------------------------
def convert_to_ascii(text):
    return unicodedata.normalize("NFKD", text).encode("ascii", "ignore").decode("ascii")


def collapse_whitespace(text):
    return re.sub(_whitespace_re, " ", text)


def expand_abbreviations(text):
    for regex, replacement in _abbreviations:
        text = re.sub(regex, replacement, text)
    return text


def basic_cleaners(text):
    return collapse_whitespace(text.lower())


def transliteration_cleaners(text):
    return collapse_whitespace(convert_to_ascii(text).lower())


def english_cleaners(text):
    text = convert_to_ascii(text).lower()
    text = normalize_numbers(text)
    text = expand_abbreviations(text)
    return collapse_whitespace(text)


_CLEANERS = {"basic_cleaners": basic_cleaners, "transliteration_cleaners": transliteration_cleaners,
             "english_cleaners": english_cleaners, "no_cleaners": lambda t: t}


def _clean(text, cleaner_names):
    for name in cleaner_names:
        if name not in _CLEANERS:
            raise Exception("Unknown cleaner: %s" % name)
        text = _CLEANERS[name](text)
    return text


def _symbols_to_sequence(syms):
    return [_symbol_to_id[s] for s in syms if s in _symbol_to_id and s not in ("_", "~")]


def text_to_sequence(text, cleaner_names):
    """Ids of the cleaned text plus the EOS id (text.py:26-53); {ARPAbet} spans are looked up
    as '@'-prefixed symbols, which this symbol table (like the reference's) does not hold."""
    seq = []
    while len(text):
        m = _curly_re.match(text)
        if not m:
            seq += _symbols_to_sequence(_clean(text, cleaner_names))
            break
        seq += _symbols_to_sequence(_clean(m.group(1), cleaner_names))
        seq += _symbols_to_sequence(["@" + s for s in m.group(2).split()])
        text = m.group(3)
    seq.append(_symbol_to_id["~"])
    return seq


def sequence_to_text(sequence):
    out = ""
    for i in sequence:
        if i in _id_to_symbol:
            s = _id_to_symbol[i]
            out += "{%s}" % s[1:] if len(s) > 1 and s[0] == "@" else s
    return out.replace("}{", " ")
